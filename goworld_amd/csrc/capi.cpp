// capi.cpp — C ABI of include/gpuaoi.h on one HIP device.
//
// Host orchestration of the per-tick pipeline (kernels in aoi.hip, sync.hip):
//   ops -> incremental grid (patch / shift / re-sort dirty cells) + mover grid
//   -> per-mover candidate bounds + scan -> diff (one wave per mover) ->
//   per-watcher scan -> own copy + mirror scatter -> segment sorts
//   [the one host sync: counts; if the event regions overflowed their
//   capacity, grow and rerun diff + events] -> reset (async).
// No neighbour lists are kept (gw_internal.hpp): collect and queries evaluate
// relations from the current grid.  No torch, no CPU fallback: every compute
// step is a HIP kernel.
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

#include "ctx.hpp"

using namespace gw;
using namespace gw::host;



namespace gw {
namespace host {

int set_err(gw_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}


// (re)allocate scratch without preserving contents; callers only grow buffers
// at points where the stream is idle (after a host sync).  An eighth of
// headroom: buffers sized by the tick's op count (which drifts by a few per
// mille between ticks in a world strip) otherwise reallocated whenever it
// reached a new high, each time a device sync plus hipFree / hipMalloc of up to
// hundreds of MB (0.3-1.2 ms on a 16M world strip)
int ensure(gw_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return 0;
    size_t nb = std::max(bytes + bytes / 8, b.cap + b.cap / 2);
    nb = (nb + 255) & ~(size_t)255;
    if (b.p) {
        HIPCHK(hipStreamSynchronize(c->st));
        HIPCHK(hipFree(b.p));
    }
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
    // pinned allocations cost ~0.16 ms per MB (hipHostMalloc 700 MB: 111 ms on
    // the box, tools/micro/pcie.hip): a quarter of headroom, so the per-tick
    // output sizes (which vary by a few %) do not reallocate every other tick
    size_t nb = std::max(bytes + bytes / 4, b.cap + b.cap / 2);
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

// a new op-dedupe session (OpLast words are tagged with it; after 2^32 - 1
// sessions the records are zeroed once and the tags restart)
int next_ol_tag(gw_ctx* c, uint32_t* tag) {
    if (++c->ol_tag == 0) {
        if (c->ol && c->slot_cap) HIPCHK(hipMemsetAsync(c->ol, 0, (size_t)c->slot_cap * sizeof(OpLast), c->st));
        c->ol_tag = 1;
    }
    *tag = c->ol_tag;
    return 0;
}

}  // namespace host
}  // namespace gw

namespace {

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


int ceil_log2(uint64_t v) {   // bits needed to represent values in [0, v)
    int b = 1;
    while (b < 63 && (1ull << b) < v) ++b;
    return b;
}

// ---- profiling ------------------------------------------------------------
// Stage events accumulate over calls until gw_get_stage_times reads them
// (after the caller's own sync), so timing adds no host sync to a tick.
constexpr size_t PROF_MAX_RECORDS = 1 << 16;   // stage records kept between collections
// prof: 0 off, 1 every stage, 2 only the dominant kernel's stage ("diff")
static bool prof_on(const gw_ctx* c, const char* name) {
    return c->prof == 1 || (c->prof == 2 && strcmp(name, "diff") == 0);
}
void prof_begin(gw_ctx* c, const char* name) {
    c->prof_cur = prof_on(c, name);
    if (!c->prof_cur || c->nstage >= PROF_MAX_RECORDS) return;
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
    if (!c->prof_cur || c->nstage >= PROF_MAX_RECORDS) return PROF_MAX_RECORDS;
    Stage& s = c->stages[c->nstage];
    s.bytes = bytes;
    (void)hipEventRecord(s.b, c->st);
    return c->nstage++;
}
void prof_set_bytes(gw_ctx* c, size_t idx, uint64_t bytes) {
    if (c->prof && idx < c->stages.size()) c->stages[idx].bytes = bytes;
}
// every recorded stage since the last collection, summed per stage name
// (one host sync and the event queries happen here, outside any timed loop)
void prof_collect(gw_ctx* c) {
    gw_stage_times& t = c->last_times;
    memset(&t, 0, sizeof t);
    if (c->nstage) (void)hipEventSynchronize(c->stages[c->nstage - 1].b);
    for (size_t i = 0; i < c->nstage; ++i) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->stages[i].a, c->stages[i].b);
        uint32_t k = 0;
        while (k < t.n && strcmp(t.name[k], c->stages[i].name) != 0) ++k;
        if (k == t.n) {
            if (t.n == GW_MAX_STAGES) continue;
            t.name[t.n++] = c->stages[i].name;
        }
        t.us[k] += ms * 1000.0;
        t.bytes_alg[k] += c->stages[i].bytes;
        t.calls[k] += 1;
    }
    c->nstage = 0;
}

// status words for scans of up to n elements (zeroed when reallocated: zero
// never matches a tag)
int ensure_scan(gw_ctx* c, uint64_t n) {
    const uint64_t tiles = (n + scan_tile() - 1) / scan_tile() + 2;
    const uint64_t bytes = tiles * scan_words() * 8;
    if (c->scan_status.cap >= bytes) return 0;
    int rc;
    if ((rc = ensure(c, c->scan_status, bytes))) return rc;
    HIPCHK(hipMemsetAsync(c->scan_status.p, 0, c->scan_status.cap, c->st));
    c->sc.status = P<unsigned long long>(c->scan_status);
    c->sc.max_tiles = c->scan_status.cap / (scan_words() * 8);
    return 0;
}

// the collect stream's scan status (sc2), as ensure_scan (cleared on growth on
// that stream, which runs every use of it)
int ensure_scan2(gw_ctx* c, uint64_t n, hipStream_t s) {
    const uint64_t tiles = (n + scan_tile() - 1) / scan_tile() + 2;
    const uint64_t bytes = tiles * scan_words() * 8;
    if (c->scan_status2.cap >= bytes) return 0;
    int rc;
    if ((rc = ensure(c, c->scan_status2, bytes))) return rc;
    HIPCHK(hipMemsetAsync(c->scan_status2.p, 0, c->scan_status2.cap, s));
    c->sc2.status = P<unsigned long long>(c->scan_status2);
    c->sc2.max_tiles = c->scan_status2.cap / (scan_words() * 8);
    c->sc2.tag = 0;
    return 0;
}

int radix_tmp(gw_ctx* c, uint64_t n_max, RadixTmp& rt) {
    uint64_t nb = (n_max + radix_tile() - 1) / radix_tile();
    if (!nb) nb = 1;
    uint64_t hn = 256 * nb;
    int rc;
    if ((rc = ensure(c, c->rs_hist, hn * 4))) return rc;
    if ((rc = ensure(c, c->rs_os, radix2_scratch(n_max) * 4 + 64))) return rc;
    if ((rc = ensure_scan(c, hn))) return rc;
    rt.hist = P<uint32_t>(c->rs_hist);
    rt.os = P<uint32_t>(c->rs_os);
    rt.sc = &c->sc;
    return 0;
}

// grow slot-indexed state to hold new_total slots, initialising the new range
int grow_slots(gw_ctx* c, uint32_t new_total) {
    if (new_total <= c->slot_cap) return 0;
    uint32_t nc = std::max<uint32_t>(new_total, c->slot_cap + c->slot_cap / 2);
    uint32_t oc = c->slot_cap;
    int rc;
    if ((rc = grow_preserve(c, c->rec, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->flags, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->gate, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->nbc, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->nbg, (size_t)oc * 4, (size_t)nc * 4))) return rc;   // read only under NBC_GATES
    if ((rc = grow_preserve(c, c->movbit, 0, (size_t)nc / 32 + 1))) return rc;
    if ((rc = grow_preserve(c, c->gmi, 0, (size_t)nc))) return rc;
    if ((rc = grow_preserve(c, c->eid_dev, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->cid_dev, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->ol, oc, nc))) return rc;     // new records: zero (session 0 is never used)
    if ((rc = grow_preserve(c, c->gnb[0], 0, nc))) return rc;    // rebuilt (grid_dirty)
    if ((rc = grow_preserve(c, c->gnb[1], 0, nc))) return rc;
    size_t n = nc - oc;
    HIPCHK(hipMemsetAsync(c->rec + oc, 0, n * sizeof(SlotRec), c->st));
    HIPCHK(hipMemsetAsync(c->flags + oc, 0, n * 4, c->st));
    HIPCHK(hipMemsetAsync(c->gate + oc, 0, n * 2, c->st));
    HIPCHK(hipMemsetAsync(c->nbc + oc, 0, n * 8, c->st));
    HIPCHK(hipMemsetAsync(c->movbit, 0, ((size_t)nc / 32 + 1) * 4, c->st));
    HIPCHK(hipMemsetAsync(c->eid_dev + oc, 0, n * 16, c->st));
    HIPCHK(hipMemsetAsync(c->cid_dev + oc, 0, n * 16, c->st));
    HIPCHK(hipMemsetAsync(c->ol + oc, 0, n * sizeof(OpLast), c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    c->slot_cap = nc;
    c->present_h.resize(nc, 0);
    c->eid_h.resize(nc, gw::host::Id16{0, 0});
    c->syncing_h.resize(nc, 0);
    c->space_of_h.resize(nc, -1);
    c->grid_dirty = true;
    return 0;
}

World world(gw_ctx* c);

// slots [base, base + n): absent, in space `sid`, every other per-slot array
// cleared (a reused range, or fresh zeros from grow_slots)
int init_space_slots(gw_ctx* c, uint32_t base, uint32_t n, uint32_t sid) {
    launch_slots_clear(world(c), c->ol, c->eid_dev, c->cid_dev, base, n, sid, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// ---- free ranges of the space lifecycle ------------------------------------
// first fit among the released ranges, else at the end (total grows); the
// caller checks the limit on the returned end before committing (commit=false
// only looks)
uint32_t take_range(std::map<uint32_t, uint32_t>& fr, uint32_t total, uint32_t n, bool commit, uint32_t* new_total) {
    for (auto it = fr.begin(); it != fr.end(); ++it)
        if (it->second >= n) {
            const uint32_t base = it->first, len = it->second;
            if (commit) {
                fr.erase(it);
                if (len > n) fr[base + n] = len - n;
            }
            *new_total = total;
            return base;
        }
    *new_total = total + n;
    return total;
}

// release [base, base + n): merged with its neighbours; a range that reaches
// the end shrinks the total instead
void give_range(std::map<uint32_t, uint32_t>& fr, uint32_t& total, uint32_t base, uint32_t n) {
    if (!n) return;
    auto nx = fr.lower_bound(base);
    if (nx != fr.end() && nx->first == base + n) {
        n += nx->second;
        nx = fr.erase(nx);
    }
    if (nx != fr.begin()) {
        auto pv = std::prev(nx);
        if (pv->first + pv->second == base) {
            base = pv->first;
            n += pv->second;
            fr.erase(pv);
        }
    }
    if (base + n == total) {
        total = base;
        // a free range may now end at the new total
        if (!fr.empty()) {
            auto last = std::prev(fr.end());
            if (last->first + last->second == total) {
                total = last->first;
                fr.erase(last);
            }
        }
    } else {
        fr[base] = n;
    }
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

// the per-field sums of the statistics shards into shard[0] (the form the
// publishing kernel writes; readers only look at shard[0])
static void fold_shards(DevStats& s) {
    for (int f = 0; f < SH_FIELDS; ++f) {
        unsigned long long t = 0;
        for (int i = 0; i < STAT_SHARDS; ++i) t += s.shard[i][f];
        s.shard[0][f] = t;
        for (int i = 1; i < STAT_SHARDS; ++i) s.shard[i][f] = 0;
    }
}

int read_stats(gw_ctx* c) {
    HIPCHK(hipMemcpyAsync(c->hstats, c->stats, sizeof(DevStats), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    fold_shards(*c->hstats);
    return 0;
}

// the collect's statistics; with a deferred tick pending, the tick's too (one
// copy of both: the tick's are final once the collect's launches are queued)
int read_cstats(gw_ctx* c) {
    const bool both = c->pt.on && !c->pt.copied;
    // one kernel writes the statistics into the pinned host buffers (coherent,
    // device-visible) and, for a deferred tick, runs its reset (which reads the
    // device statistics itself): no blit copy and no launch after the sync
    // (the reset launched after the sync instead, to overlap the host's return:
    // config #3 step +25 us)
    publish_stats(both ? &c->pt.b : nullptr, both ? (const void*)c->stats : (const void*)c->cstats,
                  both ? c->hstats_dev : c->hstats_dev + 1, (both ? 2 : 1) * sizeof(DevStats), c->st);
    if (both) c->pt.reset_queued = true;
    HIPCHK(hipStreamSynchronize(c->st));
    if (both) c->pt.copied = true;
    return 0;
}


void reset_stats_host(gw_ctx* c) { memset(c->hstats, 0, sizeof(DevStats)); }

World world(gw_ctx* c) {
    World w;
    w.cap = c->total_slots;
    w.ncells = c->total_cells;
    w.sp = c->sp_dev;
    w.rec = c->rec; w.flags = c->flags; w.gate = c->gate;
    w.gn = c->gnb[c->gcur]; w.gn_start = c->gsb[c->gcur];
    w.nbc = c->nbc;
    w.nbg = c->nbg;
    w.epoch = c->epoch;
    w.nb_u = c->nb_u;
    return w;
}

}  // namespace

World gw::host::world_of(gw_ctx* c) { return world(c); }

namespace {

// per-cell arrays for total_cells (+2); dep / arr / gm_cnt must hold zeros
// between ticks (their counters return to zero inside a tick)
int ensure_cells(gw_ctx* c) {
    const uint32_t need = c->total_cells + 2;
    if (c->cells_cap < need) {
        const uint32_t nc = std::max(need, c->cells_cap + c->cells_cap / 2);
        uint32_t** arrs[] = {&c->gsb[0], &c->gsb[1], &c->dep, &c->arr, &c->gm_cnt, &c->cnt_new, &c->dirty,
                             &c->gm_start};
        HIPCHK(hipStreamSynchronize(c->st));
        for (uint32_t** a : arrs) {
            if (*a) HIPCHK(hipFree(*a));
            *a = nullptr;
        }
        for (uint32_t** a : arrs) {
            if (hipMalloc(a, (size_t)nc * 4) != hipSuccess) {
                (void)hipGetLastError();
                c->cells_cap = 0;
                return set_err(c, GW_ENOMEM, "hipMalloc(%zu) failed", (size_t)nc * 4);
            }
        }
        c->cells_cap = nc;
        c->cells_zero = false;
        c->grid_dirty = true;
    }
    if (!c->cells_zero) {
        HIPCHK(hipMemsetAsync(c->dep, 0, (size_t)c->cells_cap * 4, c->st));
        HIPCHK(hipMemsetAsync(c->arr, 0, (size_t)c->cells_cap * 4, c->st));
        HIPCHK(hipMemsetAsync(c->gm_cnt, 0, (size_t)c->cells_cap * 4, c->st));
        c->cells_zero = true;
    }
    return 0;
}

// rebuild the current grid from the slot state (new spaces / cells)
int rebuild_grid(gw_ctx* c) {
    int rc;
    if ((rc = ensure_cells(c))) return rc;
    if (!c->grid_dirty) return 0;
    const uint32_t C = c->total_slots;
    if ((rc = ensure(c, c->k0, (size_t)C * 4)) || (rc = ensure(c, c->v0, (size_t)C * 4)) ||
        (rc = ensure(c, c->k1, (size_t)C * 4)) || (rc = ensure(c, c->v1, (size_t)C * 4)))
        return rc;
    RadixTmp rt;
    if ((rc = radix_tmp(c, C, rt))) return rc;
    reset_stats_host(c);
    HIPCHK(hipMemcpyAsync(c->stats, c->hstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
    c->stats_zero = false;
    if (C)
        grid_rebuild(world(c), c->stats, P<uint32_t>(c->k0), P<uint32_t>(c->v0), P<uint32_t>(c->k1),
                     P<uint32_t>(c->v1), rt, ceil_log2((uint64_t)c->total_cells + 1), c->st);
    else
        HIPCHK(hipMemsetAsync(c->gsb[c->gcur], 0, ((size_t)c->total_cells + 1) * 4, c->st));
    HIPCHK(hipGetLastError());
    if ((rc = read_stats(c))) return rc;
    c->h_present = c->hstats->n_present;
    c->grid_dirty = false;
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

}  // namespace

namespace gw {
namespace host {
int space_idx(gw_ctx* c, uint32_t h, uint32_t* idx) {
    const uint32_t i = h & SID_MASK;
    if (i >= c->spaces.size() || !c->spaces[i].alive) return set_err(c, GW_ERANGE, "no space %u", h);
    if ((h >> SID_BITS) != (c->spaces[i].gen & SID_GEN_MASK))
        return set_err(c, GW_ERANGE, "space id %u is stale (that space was destroyed)", h);
    *idx = i;
    return 0;
}
}  // namespace host
}  // namespace gw

// =========================================================================
extern "C" {

int gw_abi_version(void) { return GW_ABI_VERSION; }

const char* gw_last_error(const gw_ctx* c) { return c ? c->err.c_str() : "null context"; }

int gw_init(int device_id, gw_ctx** out) {
    if (!out) return GW_EINVAL;
    *out = nullptr;
    gw_ctx* c = new gw_ctx();
    c->dev = device_id;
    int rc = 0;
    do {
        if (hipSetDevice(device_id) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "hipSetDevice(%d) failed", device_id); break; }
        if (hipStreamCreateWithFlags(&c->own_st, hipStreamNonBlocking) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "stream"); break; }
        c->st = c->own_st;
        // the tick's and the collect's statistics side by side, so a collect
        // that settles a deferred tick reads both with one copy
        if (hipMalloc(&c->stats, 2 * sizeof(DevStats)) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "stats"); break; }
        // coherent: the publishing kernel writes them over PCIe (read_cstats)
        if (hipHostMalloc((void**)&c->hstats, 2 * sizeof(DevStats), hipHostMallocCoherent) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "hstats"); break; }
        if (hipHostGetDevicePointer((void**)&c->hstats_dev, c->hstats, 0) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "hstats map"); break; }
        c->cstats = c->stats + 1;
        c->hcstats = c->hstats + 1;
        if (hipMalloc(&c->scal32, 64) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "scal"); break; }
        if (hipMalloc(&c->halo, sizeof(HaloStats)) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "halo"); break; }
        (void)hipMemset(c->halo, 0, sizeof(HaloStats));
        if (hipMalloc(&c->sc.ticket, 8) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "ticket"); break; }
        (void)hipMemset(c->sc.ticket, 0, 8);
        if (hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "stream"); break; }
        if (hipEventCreateWithFlags(&c->ev_grid, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_diff, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_col, hipEventDisableTiming) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "event"); break; }
        if (hipMalloc(&c->sc2.ticket, 8) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "ticket"); break; }
        (void)hipMemset(c->sc2.ticket, 0, 8);
        memset(c->hstats, 0, 2 * sizeof(DevStats));
        (void)hipMemset(c->stats, 0, 2 * sizeof(DevStats));
        (void)hipEventCreate(&c->ev_t0);
        (void)hipEventCreate(&c->ev_t1);
        if (const char* e = getenv("GW_OVERLAP_COLLECT")) c->overlap = atoi(e) != 0;
        if (const char* e = getenv("GW_SW_HALVES")) c->sw_halves = atoi(e) != 0 ? 1 : 0;
        if (const char* e = getenv("GW_BK_FLAT")) c->bk_flat = atoi(e) != 0 ? 1 : 0;
        if (const char* e = getenv("GW_POST_SPLIT")) c->post_split = atoi(e) != 0;
        if (const char* e = getenv("GW_PLACE_SPLIT")) c->place_split = atoi(e) != 0;
        if (const char* e = getenv("GW_DIRTY_SPLIT")) c->dirty_split = atoi(e) != 0;
        if (const char* e = getenv("GW_OVERLAP_MIN")) c->overlap_min = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_CELLS_PER_D")) c->cells_per_d = std::min(4, std::max(1, atoi(e)));
        if (const char* e = getenv("GW_MOVER_WPB")) c->diff_u = atoi(e);
        if (const char* e = getenv("GW_NB_U")) c->nb_u = atoi(e);
        if (const char* e = getenv("GW_WALK_MIN")) c->walk_min = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_RANK_SORT")) c->rank_sort = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_GRID_CAP")) c->grid_cap = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_PAIR_AUTO")) c->pair_auto = atoi(e) != 0;
        if (const char* e = getenv("GW_PAIR_MAX")) {
            c->pair_max = (uint32_t)std::max(0, atoi(e));
            c->pair_auto = false;
        }
        if (const char* e = getenv("GW_MOVER_COMPACT")) c->mover_compact = atoi(e) != 0;
        if (const char* e = getenv("GW_HEAVY_MIN")) c->heavy_min = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_HEAVY_MAXM")) c->heavy_maxm = (uint32_t)std::max(0, atoi(e));
        if (const char* e = getenv("GW_DIRTY_SPAN")) c->dirty_span = (uint32_t)std::min(64, std::max(1, atoi(e)));
        if (const char* e = getenv("GW_HALF_ROWS")) c->half_rows = (uint32_t)std::min(16, std::max(0, atoi(e)));
        if (const char* e = getenv("GW_GATE_LANE_MAX")) c->gate_lane_max = (uint32_t)std::min(255, std::max(0, atoi(e)));
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
    (void)settle(c);
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    DevBuf* bufs[] = {&c->ops_buf, &c->stamp_buf, &c->pay, &c->mstat, &c->k0, &c->v0, &c->k1, &c->v1,
                      &c->gm, &c->mtmp, &c->mcell, &c->fall, &c->cand, &c->reg, &c->pidx, &c->heavy, &c->rowrec, &c->own, &c->big, &c->mir, &c->ownc, &c->mirc, &c->mlist,
                      &c->mcnt, &c->moff, &c->minfo, &c->icnt, &c->ioff, &c->mreg, &c->chunk_first, &c->srange, &c->bk_a, &c->bk_b, &c->bk_id, &c->bk_cnt, &c->bk_split, &c->ev_d, &c->rtable,
                      &c->scan_status, &c->scan_status2, &c->rs_hist, &c->rs_os,
                      &c->fbits, &c->flagged, &c->rec_cnt, &c->rec_off, &c->rec0, &c->rec1,
                      &c->gate_hist, &c->gk0, &c->gv0, &c->gk1, &c->gv1, &c->qbuf, &c->cl_slot, &c->cl_off,
                      &c->m_create.a, &c->m_create.b, &c->m_destroy.a, &c->m_destroy.b, &c->m_fanout.a,
                      &c->m_fanout.b, &c->m_flag, &c->m_at, &c->m_items, &c->m_cnt, &c->m_off};
    for (DevBuf* b : bufs) if (b->p) (void)hipFree(b->p);
    DevBuf* wb[] = {&c->wd.stamps, &c->wd.send[0], &c->wd.send[1], &c->wd.recv[0], &c->wd.recv[1], &c->wd.cnt,
                    &c->wire_d, &c->wire_tab, &c->id_up, &c->wd.ext, &c->wd.far_rows, &c->wd.far_dest,
                    &c->wd.far_cnt, &c->wd.far_sorted, &c->wd.far_off, &c->wd.far_cursor, &c->wd.far_recv,
                    &c->wd.far_mat, &c->wd.dstage};
    if (c->wire_h.p) (void)hipHostFree(c->wire_h.p);
    if (c->wd.hstage.p) (void)hipHostFree(c->wd.hstage.p);
    if (c->wd.pub_h) (void)hipHostFree(c->wd.pub_h);
    if (c->wd.staged) (void)hipEventDestroy(c->wd.staged);
    if (c->eid_dev) (void)hipFree(c->eid_dev);
    if (c->cid_dev) (void)hipFree(c->cid_dev);
    for (DevBuf* b : wb) if (b->p) (void)hipFree(b->p);
    xp_release(c);
    DevBuf* hb[] = {&c->h_enter, &c->h_leave, &c->h_rec, &c->h_cl_slot, &c->h_cl_off, &c->h_items, &c->m_create.h,
                    &c->m_destroy.h, &c->m_fanout.h};
    for (DevBuf* b : hb) if (b->p) (void)hipHostFree(b->p);
    void* ps[] = {c->halo, c->sc.ticket, c->sc2.ticket, c->movbit, c->gmi, c->rec, c->flags, c->gate, c->nbc, c->nbg, c->ol,
                  c->gnb[0], c->gnb[1], c->sp_dev, c->stats, c->scal32, c->gsb[0],
                  c->gsb[1], c->dep, c->arr, c->gm_cnt, c->cnt_new, c->dirty, c->gm_start};
    for (void* p : ps) if (p) (void)hipFree(p);
    if (c->hstats) (void)hipHostFree(c->hstats);   // hcstats lives behind it
    for (auto& s : c->stages) { (void)hipEventDestroy(s.a); (void)hipEventDestroy(s.b); }
    if (c->ev_t0) (void)hipEventDestroy(c->ev_t0);
    if (c->ev_t1) (void)hipEventDestroy(c->ev_t1);
    if (c->ev_grid) (void)hipEventDestroy(c->ev_grid);
    if (c->ev_diff) (void)hipEventDestroy(c->ev_diff);
    if (c->ev_col) (void)hipEventDestroy(c->ev_col);
    if (c->st2) {
        (void)hipStreamSynchronize(c->st2);
        (void)hipStreamDestroy(c->st2);
    }
    if (c->own_st) (void)hipStreamDestroy(c->own_st);
    delete c;
}

int gw_space_create(gw_ctx* c, float aoi_dist, uint32_t capacity, const float* bounds, uint32_t* space_id,
                    uint32_t* slot_base) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    if (!(aoi_dist > 0) || !std::isfinite(aoi_dist))
        return set_err(c, GW_EINVAL, "defaultAOIDistance <= 0");          // Space.go:92-94
    if (capacity == 0) return set_err(c, GW_EINVAL, "capacity must be > 0");
    if (!c->segs.empty()) return set_err(c, GW_ESTATE, "space create with ops pending: tick first");
    float b[4] = {-1000.f, -1000.f, 1000.f, 1000.f};                       // Space.GetSpaceRange, Space.go:52-54
    if (bounds) for (int i = 0; i < 4; ++i) b[i] = bounds[i];
    if (!(b[2] > b[0]) || !(b[3] > b[1]) || !std::isfinite(b[0]) || !std::isfinite(b[1]) || !std::isfinite(b[2]) ||
        !std::isfinite(b[3]))
        return set_err(c, GW_EINVAL, "bad bounds");
    // square cells of side >= d / cells_per_d; at most 4096 cells per axis (a
    // space's cells then fit the 25 cell bits of a grid entry); a
    // search window (2d plus the rounding margin of dev_common.hpp
    // search_rect) spans at most 11 rows, so a mover's two windows fit the
    // 32 row ranges of one wave (Flat)
    double ex = (double)b[2] - b[0], ez = (double)b[3] - b[1];
    double maxabs = std::max(std::max(std::fabs((double)b[0]), std::fabs((double)b[2])),
                             std::max(std::fabs((double)b[1]), std::fabs((double)b[3])));
    double span = 2.0 * aoi_dist + 4e-6 * (maxabs + aoi_dist) + 1e-3;
    double cs = std::max((double)aoi_dist / c->cells_per_d, std::max(ex, ez) / 4096.0);
    cs = std::max(cs, span / 9.0);
    SpaceHost s{};
    s.d = aoi_dist;
    s.cap = capacity;
    s.alive = true;
    s.p.d = aoi_dist;
    s.p.x0 = b[0];
    s.p.z0 = b[1];
    s.p.inv_cs = (float)(1.0 / cs);
    s.p.W = std::max(1, (int)std::ceil(ex / cs));
    s.p.H = std::max(1, (int)std::ceil(ez / cs));
    s.p.alive = 1;
    s.p.own_lo = -INFINITY;
    s.p.own_hi = INFINITY;
    uint64_t ncells = (uint64_t)s.p.W * (uint64_t)s.p.H;
    if (ncells >= CELL_MASK) return set_err(c, GW_ERANGE, "too many grid cells");
    // slot and cell ranges: a released range first (first fit), else at the end
    uint32_t nt_slots = 0, nt_cells = 0;
    const uint32_t base = take_range(c->free_slots, c->total_slots, capacity, false, &nt_slots);
    const uint32_t cbase = take_range(c->free_cells, c->total_cells, (uint32_t)ncells, false, &nt_cells);
    if ((uint64_t)base + capacity >= (1ull << 31) || (uint64_t)nt_slots >= (1ull << 31))
        return set_err(c, GW_ERANGE, "too many slots");
    if ((uint64_t)cbase + ncells + 1 > CELL_MASK || (uint64_t)nt_cells + 1 > CELL_MASK)
        return set_err(c, GW_ERANGE, "too many grid cells");
    int rc;
    if ((rc = grow_slots(c, nt_slots))) return rc;
    // a destroyed space's id is handed out again (lowest first)
    uint32_t sid = 0;
    while (sid < c->spaces.size() && c->spaces[sid].alive) ++sid;
    if (sid > SID_MASK) return set_err(c, GW_ERANGE, "too many spaces");
    if (sid < c->spaces.size()) s.gen = c->spaces[sid].gen;   // the destroyed space's next generation
    if ((rc = init_space_slots(c, base, capacity, sid))) return rc;
    (void)take_range(c->free_slots, c->total_slots, capacity, true, &nt_slots);
    (void)take_range(c->free_cells, c->total_cells, (uint32_t)ncells, true, &nt_cells);
    c->total_slots = nt_slots;
    c->total_cells = nt_cells;
    s.base = base;
    s.p.cell_base = cbase;
    if (sid == c->spaces.size()) c->spaces.push_back(s);
    else c->spaces[sid] = s;
    c->grid_dirty = true;
    for (uint32_t i = 0; i < capacity; ++i) {
        c->space_of_h[base + i] = (int32_t)sid;
        c->present_h[base + i] = 0;
    }
    if ((rc = upload_spaces(c))) return rc;
    if (space_id) *space_id = sid_handle(c->spaces[sid], sid);
    if (slot_base) *slot_base = base;
    return 0;
}

int gw_space_restore(gw_ctx* c, uint32_t sid_h, const uint32_t* slots, const float* x, const float* y,
                     const float* z, const float* yaw, uint32_t n, uint8_t sync_flags) {
    if (!c || (n && (!slots || !x || !y || !z || !yaw))) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    uint32_t sid = 0;
    if (int rs = space_idx(c, sid_h, &sid)) return rs;
    if (!c->segs.empty()) return set_err(c, GW_ESTATE, "restore with ops pending: tick first");
    if (!n) return 0;
    const SpaceHost& sp = c->spaces[sid];
    std::vector<uint8_t> seen;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = slots[i];
        if (s < sp.base || s >= sp.base + sp.cap)
            return set_err(c, GW_ERANGE, "restore %u: slot %u not in space %u", i, s, sid);
        if (!(std::isfinite(x[i]) && std::isfinite(z[i])))
            return set_err(c, GW_EINVAL, "restore %u: non-finite coordinates", i);
        if (seen.empty()) seen.assign(sp.cap, 0);
        if (seen[s - sp.base]++ || (c->validate && c->present_h[s]))
            return set_err(c, GW_ESTATE, "restore %u: slot %u already in the space", i, s);
    }
    int rc;
    std::vector<float4> p(n);
    for (uint32_t i = 0; i < n; ++i) p[i] = make_float4(x[i], y[i], z[i], yaw[i]);
    const size_t off = ((size_t)n * 4 + 15) & ~(size_t)15;     // float4 payload after the slots
    if ((rc = ensure(c, c->qbuf, off + (size_t)n * 16))) return rc;
    uint32_t* dslots = P<uint32_t>(c->qbuf);
    float4* dp = (float4*)(P<uint8_t>(c->qbuf) + off);
    HIPCHK(hipMemcpyAsync(dslots, slots, (size_t)n * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(dp, p.data(), (size_t)n * 16, hipMemcpyHostToDevice, c->st));
    launch_restore(world(c), dslots, dp, n, c->stamp_base, sync_flags, c->st);
    c->flag_bound += n;
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));            // the host arrays are the caller's
    c->stamp_base += n;
    for (uint32_t i = 0; i < n; ++i) c->present_h[slots[i]] = 1;
    ++c->epoch;                                      // neighbour counts cached by the diff are stale
    c->grid_dirty = true;                            // rebuilt (one radix sort) before the next use
    return 0;
}

// entities present in a space's slot range, counted on the device (after
// device-resident submits the host mirror is not exact)
static int count_present(gw_ctx* c, uint32_t base, uint32_t n, uint64_t* out) {
    HIPCHK(hipMemsetAsync(c->scal32, 0, 8, c->st));
    launch_count_present(c->rec, base, n, (unsigned long long*)c->scal32, c->st);
    HIPCHK(hipGetLastError());
    unsigned long long v = 0;
    HIPCHK(hipMemcpyAsync(&v, c->scal32, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    *out = v;
    return 0;
}

// host mirrors of slots [base, base + n) -> nothing (released) or -> [to, to + n) (moved)
static void move_host_slots(gw_ctx* c, uint32_t base, uint32_t n, int64_t to) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = base + i;
        const gw::host::Id16 id = c->eid_h[s];
        if (to >= 0) {
            const uint32_t d = (uint32_t)to + i;
            c->present_h[d] = c->present_h[s];
            c->eid_h[d] = id;
            c->syncing_h[d] = c->syncing_h[s];
            if (id.a | id.b) c->id_slot[id] = d;
        } else if (id.a | id.b) {
            auto it = c->id_slot.find(id);
            if (it != c->id_slot.end() && it->second == s) c->id_slot.erase(it);
        }
        c->present_h[s] = 0;
        c->eid_h[s] = gw::host::Id16{0, 0};
        c->syncing_h[s] = 0;
        c->space_of_h[s] = -1;
    }
}

// Space.OnDestroy destroys every entity first (Space.go:143-151: each
// Destroy is a Space.leave -> aoiMgr.Leave, ticked before this call), then
// SpaceManager.delSpace (SpaceManager.go:25-27).  Always checked on the
// device: destroying a space that still holds an entity is an error.  Its
// slot and cell ranges are cleared (pending sync flags of entities that left
// it into the nil space go with them: collect first) and reused.
int gw_space_destroy(gw_ctx* c, uint32_t sid_h) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    uint32_t sid = 0;
    if (int rs = space_idx(c, sid_h, &sid)) return rs;
    if (!c->segs.empty()) return set_err(c, GW_ESTATE, "space destroy with ops pending: tick first");
    SpaceHost& s = c->spaces[sid];
    if (c->wd.on && sid == c->wd.sid) return set_err(c, GW_ESTATE, "space %u is the context's world strip", sid);
    uint64_t np = 0;
    int rc;
    if ((rc = count_present(c, s.base, s.cap, &np))) return rc;
    if (np) return set_err(c, GW_ESTATE, "space %u not empty (%llu entities)", sid, (unsigned long long)np);
    launch_slots_clear(world(c), c->ol, c->eid_dev, c->cid_dev, s.base, s.cap, sid, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    move_host_slots(c, s.base, s.cap, -1);
    give_range(c->free_slots, c->total_slots, s.base, s.cap);
    give_range(c->free_cells, c->total_cells, s.p.cell_base, (uint32_t)(s.p.W * s.p.H));
    s.alive = false;
    s.p.alive = 0;
    ++s.gen;
    c->grid_dirty = true;
    ++c->epoch;
    return upload_spaces(c);
}

// Space.enter adds entities without bound (Space.go:179-217): capacity grows
// in place when the slots behind the space are free, else the space's state
// moves to a new range (its slots change: new_base; events and records of
// later calls carry the new slots).  No ops may be pending.
int gw_space_grow(gw_ctx* c, uint32_t sid_h, uint32_t new_capacity, uint32_t* new_base) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    uint32_t sid = 0;
    if (int rs = space_idx(c, sid_h, &sid)) return rs;
    if (!c->segs.empty()) return set_err(c, GW_ESTATE, "space grow with ops pending: tick first");
    SpaceHost& s = c->spaces[sid];
    if (new_capacity < s.cap) return set_err(c, GW_EINVAL, "capacity %u below the current %u", new_capacity, s.cap);
    if (new_base) *new_base = s.base;
    if (new_capacity == s.cap) return 0;
    const uint32_t delta = new_capacity - s.cap, end = s.base + s.cap;
    int rc;
    // in place: the space is last, or a released range starts right behind it
    auto nx = c->free_slots.find(end);
    const bool at_end = end == c->total_slots;
    if (at_end || (nx != c->free_slots.end() && nx->second >= delta)) {
        if ((uint64_t)end + delta >= (1ull << 31)) return set_err(c, GW_ERANGE, "too many slots");
        if (at_end) {
            if ((rc = grow_slots(c, end + delta))) return rc;
        }
        if ((rc = init_space_slots(c, end, delta, sid))) return rc;
        if (at_end) {
            c->total_slots = end + delta;
        } else {
            const uint32_t len = nx->second;
            c->free_slots.erase(nx);
            if (len > delta) c->free_slots[end + delta] = len - delta;
        }
        for (uint32_t i = 0; i < delta; ++i) c->space_of_h[end + i] = (int32_t)sid;
        s.cap = new_capacity;
        c->grid_dirty = true;
        return 0;
    }
    if (c->wd.on && sid == c->wd.sid)
        return set_err(c, GW_ESTATE, "a world strip keeps slot = entity id: it cannot move (grow it in place)");
    uint32_t nt = 0;
    const uint32_t nb = take_range(c->free_slots, c->total_slots, new_capacity, false, &nt);
    if ((uint64_t)nb + new_capacity >= (1ull << 31) || (uint64_t)nt >= (1ull << 31))
        return set_err(c, GW_ERANGE, "too many slots");
    if ((rc = grow_slots(c, nt))) return rc;
    (void)take_range(c->free_slots, c->total_slots, new_capacity, true, &nt);
    c->total_slots = nt;
    const World w = world(c);
    launch_slots_clear(w, c->ol, c->eid_dev, c->cid_dev, nb + s.cap, delta, sid, c->st);
    launch_slots_move(w, c->ol, c->eid_dev, c->cid_dev, s.base, nb, s.cap, c->st);
    launch_slots_clear(w, c->ol, c->eid_dev, c->cid_dev, s.base, s.cap, sid, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    const uint32_t ob = s.base, oc = s.cap;
    move_host_slots(c, ob, oc, nb);
    for (uint32_t i = 0; i < new_capacity; ++i) c->space_of_h[nb + i] = (int32_t)sid;
    give_range(c->free_slots, c->total_slots, ob, oc);
    s.base = nb;
    s.cap = new_capacity;
    c->grid_dirty = true;
    ++c->epoch;
    if (new_base) *new_base = nb;
    return 0;
}

int gw_context_info(gw_ctx* c, gw_ctx_info* out) {
    if (!c || !out) return GW_EINVAL;
    memset(out, 0, sizeof *out);
    out->total_slots = c->total_slots;
    out->total_cells = c->total_cells;
    for (auto& sp : c->spaces)
        if (sp.alive) {
            ++out->live_spaces;
            out->live_slots += sp.cap;
            out->live_cells += (uint32_t)(sp.p.W * sp.p.H);
        }
    return 0;
}

int gw_submit(gw_ctx* c, const gw_op* ops, uint32_t n) {
    if (!c || (!ops && n)) return GW_EINVAL;
    if (!n) return 0;
    if (c->validate) {
        int rc = validate_ops(c, ops, n);
        if (rc) return rc;
    }
    OpSeg sg{true, nullptr, nullptr, n, c->pend_host.size(), nullptr};
    c->pend_host.insert(c->pend_host.end(), ops, ops + n);
    c->segs.push_back(sg);
    return 0;
}

int gw_submit_device(gw_ctx* c, const gw_op* dev_ops, uint32_t n) {
    if (!c || (!dev_ops && n)) return GW_EINVAL;
    if (!n) return 0;
    c->validate = false;   // device-resident ops are trusted; the host mirror is no longer exact
    c->segs.push_back(OpSeg{false, dev_ops, nullptr, n, 0, nullptr});
    return 0;
}

int gw_submit_device_stamped(gw_ctx* c, const gw_op* dev_ops, const uint64_t* dev_stamps, uint32_t n) {
    if (!c || ((!dev_ops || !dev_stamps) && n)) return GW_EINVAL;
    if (!n) return 0;
    c->validate = false;
    c->segs.push_back(OpSeg{false, dev_ops, dev_stamps, n, 0, nullptr});
    return 0;
}

int gw_submit_device_rows(gw_ctx* c, const gw_halo_row* dev_rows, uint32_t n) {
    if (!c || (!dev_rows && n)) return GW_EINVAL;
    if (!n) return 0;
    c->validate = false;
    c->segs.push_back(OpSeg{false, nullptr, nullptr, n, 0, dev_rows});
    return 0;
}

int gw_route_halo(gw_ctx* c, const gw_op* dev_ops, const uint64_t* dev_stamps, uint32_t n, float max_step,
                  const gw_halo_dst* dsts, uint32_t n_dst) {
    if (!c || (n && (!dev_ops || !dev_stamps)) || (n_dst && !dsts)) return GW_EINVAL;
    if (n_dst > 2) return set_err(c, GW_EINVAL, "at most 2 halo destinations");
    if (int rs = settle(c)) return rs;
    if (!(max_step >= 0)) return set_err(c, GW_EINVAL, "max_step must be >= 0");
    (void)hipSetDevice(c->dev);
    HaloDsts D{};
    D.n = n_dst;
    for (uint32_t d = 0; d < n_dst; ++d) {
        if (!dsts[d].rows && dsts[d].cap_entities) return GW_EINVAL;
        D.d[d] = HaloDst{dsts[d].x_lo, dsts[d].x_hi, dsts[d].rows, dsts[d].cap_entities};
    }
    if (!c->total_slots) return set_err(c, GW_EINVAL, "no space");
    // n == 0 still runs: the buffers must become all NOPs
    int rc;
    uint32_t tag = 0;
    if ((rc = next_ol_tag(c, &tag))) return rc;
    launch_route_halo(world(c), dev_ops, (const unsigned long long*)dev_stamps, n, max_step, D, c->ol, tag,
                      c->halo, c->st);
    HIPCHK(hipGetLastError());
    return 0;
}

int gw_halo_status(gw_ctx* c, uint64_t* overflow, uint64_t* long_moves, uint64_t* bad_ops) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    HaloStats h{};
    HIPCHK(hipMemcpyAsync(&h, c->halo, sizeof h, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemsetAsync(c->halo, 0, sizeof h, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (overflow) *overflow = h.overflow;
    if (long_moves) *long_moves = h.long_moves;
    if (bad_ops) *bad_ops = h.bad_ops;
    return 0;
}

int gw_space_set_ownership(gw_ctx* c, uint32_t sid_h, float x_lo, float x_hi) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    uint32_t sid = 0;
    if (int rs = space_idx(c, sid_h, &sid)) return rs;
    if (!(x_lo < x_hi)) return set_err(c, GW_EINVAL, "empty ownership range");
    c->spaces[sid].p.own_lo = x_lo;
    c->spaces[sid].p.own_hi = x_hi;
    return upload_spaces(c);
}

int gw_set_clients(gw_ctx* c, const uint32_t* slots, const uint16_t* gates, uint32_t n) {
    if (!c || (n && (!slots || !gates))) return GW_EINVAL;
    if (!n) return 0;
    if (int rs = settle(c)) return rs;
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
    ++c->epoch;   // neighbour-with-client counts cached by the last tick are stale
    launch_set_clients(world(c), P<uint32_t>(c->gk0), (const uint16_t*)c->gv0.p, n, !c->grid_dirty, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

static int ensure_events(gw_ctx* c) {
    int r;
    if ((r = ensure(c, c->own, c->own_cap * 4)) || (r = ensure(c, c->mir, c->own_cap * 8)) ||
        (r = ensure(c, c->bk_a, c->ev_cap * 8)) || (r = ensure(c, c->bk_b, c->ev_cap * 8)) ||
        (r = ensure(c, c->bk_id, c->ev_cap * 2)) ||
        (r = ensure(c, c->ev_d, c->ev_cap * sizeof(gw_event))) ||
        (r = ensure(c, c->chunk_first, (c->ev_cap / 64 + 1) * 4)) ||
        (r = ensure(c, c->rtable, radix2_scratch(c->ev_cap) * 4 + 64)))
        return r;
    const uint64_t tiles = (c->ev_cap + BK_TILE - 1) / BK_TILE;
    if ((r = ensure(c, c->bk_cnt, (tiles << BK_MAXBITS) * 8)) || (r = ensure_scan(c, tiles << BK_MAXBITS)) ||
        (r = ensure(c, c->bk_split, BK_NSPLIT * 4)))
        return r;
    return 0;
}

// buckets for the expected event count: mean about BK_MEAN; the general sort
// when even the most buckets would average over BK_LCAP / 2, or for a while
// after a bucket overflowed
static void choose_buckets(gw_ctx* c, TickBufs& b, bool full = false) {
    // items (own runs + mirror events) of the last tick, else about half the events
    const uint64_t est = std::max<uint64_t>(c->it_est ? c->it_est : c->ev_est / 2, 1);
    b.it_hint = est;
    int bits = 1;
    while (bits < BK_MAXBITS && (est >> bits) > BK_MEAN) ++bits;
    bits = std::min(bits, b.wbits + 1);
    b.bk_bits = bits;
    b.ev_full = full || c->ev_full_ticks > 0 || (est >> bits) > (uint64_t)BK_LCAP / 2 || b.wbits > BK_MAX_WBITS;
}

// small-space mode: every space's grid (entries + row starts of both grids)
// fits in SMALL_LDS_MAX bytes of LDS, and there are many spaces
static void small_mode(gw_ctx* c, TickBufs& b) {
    uint32_t me = 0, mc = 0;
    for (auto& sp : c->spaces)
        if (sp.alive) {
            me = std::max(me, sp.cap);
            mc = std::max(mc, (uint32_t)(sp.p.W * sp.p.H));
        }
    static const bool on = !getenv("GW_SMALL") || atoi(getenv("GW_SMALL")) != 0;
    b.n_spaces = (uint32_t)c->spaces.size();
    const bool small = on && b.n_spaces >= 2 && (size_t)me * sizeof(GEnt) + 2 * ((size_t)mc + 1) * 4 <= SMALL_LDS_MAX;
    b.small_ents = small ? me : 0;
    b.small_cells = small ? mc : 0;
    static const bool halves = !getenv("GW_MOVER_HALVES") || atoi(getenv("GW_MOVER_HALVES")) != 0;
    b.small_halves = halves ? 1 : 0;
}

static void bind_events(gw_ctx* c, TickBufs& b) {
    b.own_cap = c->own_cap;
    b.own = P<uint32_t>(c->own); b.mir = P<uint64_t>(c->mir);
    b.bk_a = P<uint64_t>(c->bk_a); b.bk_b = P<uint64_t>(c->bk_b);
    b.fk0 = P<uint32_t>(c->bk_a); b.fv0 = b.fk0 + c->ev_cap;
    b.fk1 = P<uint32_t>(c->bk_b); b.fv1 = b.fk1 + c->ev_cap;
    b.bk_cnt = P<unsigned long long>(c->bk_cnt);
    b.bk_id = P<uint16_t>(c->bk_id);
    b.bk_split = P<uint32_t>(c->bk_split);
    b.bk_tiles = (uint32_t)((c->ev_cap + BK_TILE - 1) / BK_TILE);
    b.ev = P<gw_event>(c->ev_d);
    b.chunk_first = P<uint32_t>(c->chunk_first);
    b.ev_cap = c->ev_cap;
    b.rtable = P<uint32_t>(c->rtable);
}

// Second half of a tick: read the statistics (one host sync, or none when a
// collect has just synced the stream), redo diff + events if the own-event
// regions overflowed, reset the per-op state, fill the outputs.
static int finish_tick(gw_ctx* c, gw_tick_out* out) {
    auto& p = c->pt;
    if (!p.on) {
        if (out) *out = c->last_out;
        return 0;
    }
    p.on = false;
    (void)hipSetDevice(c->dev);
    TickBufs b = p.b;
    const uint32_t M = p.M, NC = p.NC, flags = p.flags;
    size_t s_grid = p.s_grid, s_movers = p.s_movers, s_diff = p.s_diff, s_events = p.s_events;
    int rc;
    if (p.copied) HIPCHK(hipStreamSynchronize(c->st));
    else if ((rc = read_stats(c))) return rc;
    // the own-event regions or the event buffers did not fit: grow to the
    // exact bounds and rerun diff + events (their inputs are intact; the mover
    // bitmap was cleared by the list pass).  A region overflow hides the events
    // of the movers it stopped, so the event count is only exact on the next
    // attempt: up to three.
    bool redone = false;
    for (int attempt = 0; c->hstats->overflow; ++attempt) {
        redone = true;
        if (attempt == 3) return set_err(c, GW_ENOMEM, "event buffers overflowed three times");
        const uint64_t E = (c->hstats->ev_pk & 0xffffffffull) + (c->hstats->ev_pk >> 32);
        const uint64_t ct = c->hstats->cand_total & CAND_MASK;
        if (ct > c->own_cap) c->own_cap = ct + ct / 4 + 4096;
        if (E > c->ev_cap) c->ev_cap = E + E / 4 + 4096;
        // a bucket outgrew the LDS sort: this attempt on the general sort (its
        // output gives the next tick quantile bounds); twice running, the
        // general sort for a while
        const bool bk_over = c->hstats->bk_max != 0;
        if (bk_over && ++c->bk_overflows >= 2) c->ev_full_ticks = 16;
        c->ev_est = std::max(c->ev_est, E);
        if ((rc = ensure_events(c))) return rc;
        bind_events(c, b);
        choose_buckets(c, b, bk_over || b.ev_full);
        DevStats* h = c->hstats;
        h->overflow = 0; h->n_big = 0; h->ev_pk = 0; h->n_mlist = 0; h->n_fall = 0; h->n_conflicts = 0; h->n_sort = 0; h->bk_max = 0; h->n_items = 0; h->bk_tiles = 0; h->bk_cells = 0;
        for (int i = 0; i < STAT_SHARDS; ++i)      // the diff's shards restart; the mover count (its
            for (int f = 0; f < SH_FIELDS; ++f)      // total in shard[0]) stays
                if (f != SH_MOVERS || i) h->shard[i][f] = 0;
        HIPCHK(hipMemcpyAsync(c->stats, c->hstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
        prof_begin(c, "diff");
        tick_diff(b, c->st);
        s_diff = prof_end(c, 0);
        prof_begin(c, "events");
        tick_events(b, c->sc, c->st);
        s_events = prof_end(c, 0);
        HIPCHK(hipGetLastError());
        if ((rc = read_stats(c))) return rc;
    }
    if (!p.reset_queued || redone) {                 // (a collect queued it behind its statistics copy)
        prof_begin(c, "reset");
        tick_reset(b, c->st);                        // asynchronous: the next call orders behind it
        prof_end(c, (uint64_t)M * 24);
    }
    p.reset_queued = false;
    c->stats_zero = true;                            // the reset zeroed the device statistics
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    HIPCHK(hipGetLastError());
    DevStats& hs = *c->hstats;
    c->h_present = hs.n_present;
    if (c->wd.on) c->wd.conflicts_acc += hs.n_conflicts;   // the final attempt's count (gw_world_status)
    gw_tick_out o{};
    const uint64_t n_enter = hs.ev_pk & 0xffffffffull, n_leave = hs.ev_pk >> 32;
    if (!(flags & GW_TICK_NO_EVENTS)) {                // sizes the next tick's buckets
        c->ev_est = n_enter + n_leave;
        if (!b.ev_full) c->it_est = hs.n_items;
        // the launches of the event stage (flatten chunks, bucket tiles) scale
        // with ev_cap: after a burst, come back down to twice the need (the
        // buffers keep their size; an overflow grows it again)
        const uint64_t want = std::max<uint64_t>(48ull * M + 4096, 2 * (n_enter + n_leave) + 4096);
        if (c->ev_cap > 2 * want) c->ev_cap = want;
    }
    if (c->ev_full_ticks > 0) --c->ev_full_ticks;
    if (!b.ev_full) c->bk_overflows = 0;
    uint64_t n_mov = 0;
    n_mov = hs.shard[0][SH_MOVERS];                  // shard[0] holds the totals (fold_shards / the publish)
    // candidates tested == the candidate bounds; a_old | a_new << 32 per shard
    const uint64_t pairs = hs.cand_total & CAND_MASK;
    uint64_t a_old = 0, a_new = 0;
    a_old = hs.shard[0][SH_AOLD] & 0xffffffffull;
    a_new = hs.shard[0][SH_AOLD] >> 32;
    if (getenv("GW_DEBUG_STATS")) {
        unsigned long long f0 = 0, f2 = 0;
        f0 = hs.shard[0][0];
        f2 = hs.shard[0][2];
        fprintf(stderr, "gw_tick: movers %llu gm %llu cand %llu ev %llu+%llu big %llu mlist %llu "
                "f0 %llu f2 %llu bits %d full %d items %llu\n",
                (unsigned long long)n_mov, hs.n_gm, hs.cand_total & CAND_MASK, hs.ev_pk & 0xffffffffull,
                hs.ev_pk >> 32, hs.n_big, hs.n_mlist, f0, f2, b.bk_bits, b.ev_full, hs.n_items);
    }
    o.ops = M;
    o.movers = n_mov;
    o.pairs_tested = pairs;
    if (!(flags & GW_TICK_NO_EVENTS) && n_mov) c->cand_mean = n_mov >= gw_ctx::PAIR_MOVERS ? pairs / n_mov : ~0ull;
    o.nbr_old = a_old;
    o.nbr_new = a_new;
    o.enter_dev = (flags & GW_TICK_NO_EVENTS) ? nullptr : P<gw_event>(c->ev_d);
    o.leave_dev = (flags & GW_TICK_NO_EVENTS) ? nullptr : P<gw_event>(c->ev_d) + (hs.ev_pk & 0xffffffffull);
    o.n_enter = n_enter;
    o.n_leave = n_leave;
    // SURVEY 8(d) algorithmic bytes of the AOI part (records are counted by gw_sync_collect)
    const uint64_t n_evt = n_enter + n_leave;
    o.bytes_alg = 20ull * n_mov + 8ull * hs.n_present + 4ull * (a_old + a_new) + 8ull * n_evt;
    if (c->prof) {
        // grid: entries moved (16 B read + 16 B written + 4 B index) + per-cell counts (16 B)
        prof_set_bytes(c, s_grid, 36ull * hs.n_present + 16ull * NC);
        prof_set_bytes(c, s_movers, 40ull * hs.n_gm);
        // diff: candidates (16 B grid / 32 B mover grid; counted at 16 B) + own events (4 B)
        prof_set_bytes(c, s_diff, 16ull * pairs + 4ull * n_evt);
        // events: per-watcher counts and offsets (16 B per slot) + events (8 B) + own copies (4 B)
        // events: flatten (read 4-8 B, write 8 B) + three sort passes (read 12 B, write 8 B) per event
        prof_set_bytes(c, s_events, 76ull * n_evt);
    }
    if ((flags & GW_TICK_COPY_TO_HOST) && !(flags & GW_TICK_NO_EVENTS)) {
        if ((rc = ensure_host(c, c->h_enter, std::max<uint64_t>(n_enter, 1) * sizeof(gw_event)))) return rc;
        if ((rc = ensure_host(c, c->h_leave, std::max<uint64_t>(n_leave, 1) * sizeof(gw_event)))) return rc;
        if (n_enter) HIPCHK(hipMemcpyAsync(c->h_enter.p, c->ev_d.p, n_enter * sizeof(gw_event), hipMemcpyDeviceToHost, c->st));
        if (n_leave)
            HIPCHK(hipMemcpyAsync(c->h_leave.p, P<gw_event>(c->ev_d) + n_enter, n_leave * sizeof(gw_event),
                                  hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        o.enter = (const gw_event*)c->h_enter.p;
        o.leave = (const gw_event*)c->h_leave.p;
    }
    float ms = 0;
    if (flags & GW_TICK_COPY_TO_HOST) {                // synced above: the span is known
        HIPCHK(hipEventSynchronize(c->ev_t1));
        (void)hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1);
    }
    o.device_us = ms * 1000.0;
    c->last_out = o;
    if (out) *out = o;
    if (hs.bad_ops) return set_err(c, GW_EINVAL, "%llu ops with bad slot/kind (ignored)", hs.bad_ops);
    return 0;
}

}  // extern "C"

namespace gw {
namespace host {
int settle(gw_ctx* c) { return finish_tick(c, nullptr); }
}  // namespace host
}  // namespace gw

extern "C" {



int gw_tick(gw_ctx* c, uint32_t flags, gw_tick_out* out) {
    if (!c || !out) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    memset(out, 0, sizeof *out);
    int rc0 = settle(c);                             // a deferred tick before this one
    if (rc0) return rc0;
    c->wd.submitted = false;
    bool host_ops = false;                           // pageable host ops: no deferral
    for (auto& sg : c->segs) host_ops |= sg.host;
    uint64_t M64 = 0;
    for (auto& s : c->segs) M64 += s.n;
    if (M64 >= (1ull << 30)) return set_err(c, GW_ERANGE, "too many ops in one tick");
    const uint32_t M = (uint32_t)M64;
    const uint32_t C = c->total_slots;
    int rc;
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    ++c->epoch;
    if (M == 0 || C == 0) {
        c->segs.clear();
        c->pend_host.clear();
        return 0;
    }
    if ((rc = rebuild_grid(c))) return rc;           // the pre-tick grid (syncs only when dirty)
    // ---- the tick's op stream, in submission order -----------------------
    const gw_op* ops = nullptr;
    const unsigned long long* stamps = nullptr;
    bool any_stamped = false, all_stamped = true;
    for (auto& s : c->segs) {
        any_stamped |= s.stamps != nullptr || s.rows != nullptr;
        all_stamped &= s.stamps != nullptr || s.rows != nullptr;
    }
    if (any_stamped && !all_stamped) {
        c->segs.clear();
        c->pend_host.clear();
        return set_err(c, GW_EINVAL, "a tick mixes stamped and unstamped ops");
    }
    if (c->segs.size() == 1 && !c->segs[0].host && !c->segs[0].rows) {
        ops = c->segs[0].dev;
        stamps = (const unsigned long long*)c->segs[0].stamps;
    } else {
        if ((rc = ensure(c, c->ops_buf, (size_t)M * sizeof(gw_op)))) return rc;
        if (any_stamped && (rc = ensure(c, c->stamp_buf, (size_t)M * 8))) return rc;
        size_t off = 0;
        bool all_dev = c->segs.size() <= (size_t)SEG_MAX;
        for (auto& s : c->segs) all_dev &= !s.host && (!any_stamped || s.rows || s.stamps);
        if (all_dev) {                               // one launch for every segment
            SegTable t{};
            for (auto& s : c->segs) {
                t.seg[t.n] = SegTable::Seg{s.dev, (const unsigned long long*)s.stamps, s.rows, (uint32_t)off};
                ++t.n;
                off += s.n;
            }
            t.total = (uint32_t)off;
            launch_gather_segs(t, P<gw_op>(c->ops_buf), any_stamped ? P<unsigned long long>(c->stamp_buf) : nullptr,
                               c->st);
        }
        for (auto& s : c->segs) {
            if (all_dev) break;
            if (s.rows)
                launch_split_rows(s.rows, s.n, P<gw_op>(c->ops_buf) + off, P<unsigned long long>(c->stamp_buf) + off,
                                  c->st);
            else if (s.host)
                HIPCHK(hipMemcpyAsync(P<gw_op>(c->ops_buf) + off, c->pend_host.data() + s.host_off,
                                      (size_t)s.n * sizeof(gw_op), hipMemcpyHostToDevice, c->st));
            else
                HIPCHK(hipMemcpyAsync(P<gw_op>(c->ops_buf) + off, s.dev, (size_t)s.n * sizeof(gw_op),
                                      hipMemcpyDeviceToDevice, c->st));
            if (s.stamps)
                HIPCHK(hipMemcpyAsync(P<uint64_t>(c->stamp_buf) + off, s.stamps, (size_t)s.n * 8,
                                      hipMemcpyDeviceToDevice, c->st));
            off += s.n;
        }
        ops = P<gw_op>(c->ops_buf);
        if (any_stamped) stamps = P<unsigned long long>(c->stamp_buf);
    }
    const uint32_t NC = c->total_cells;
    const uint64_t M2 = 2ull * M;
    c->flag_bound += M;                              // an op may flag its slot
    // ---- buffers (event regions sized from the last tick; grown on overflow)
    // a NO_EVENTS tick (bulk load / restore path) only updates the state: no
    // diff, no event stage, and its op count does not size the event buffers
    const bool ev_on = !(flags & GW_TICK_NO_EVENTS);
    if (ev_on) {
        c->own_cap = std::max<uint64_t>(c->own_cap, 64ull * M + 4096);
        c->ev_cap = std::max<uint64_t>(c->ev_cap, 48ull * M + 4096);
    }
    if ((rc = ensure(c, c->gm, M2 * sizeof(MEnt))) || (rc = ensure(c, c->mtmp, (size_t)M * sizeof(MEnt))) ||
        (rc = ensure(c, c->mcell, (size_t)M * 16)) ||
        (rc = ensure(c, c->cand, M2 * 8)) || (rc = ensure(c, c->reg, M2 * 8)) ||
        (rc = ensure(c, c->ownc, M2 * 8)) || (rc = ensure(c, c->mirc, M2 * 8)) || (rc = ensure(c, c->big, M2 * 4)) ||
        (rc = ensure(c, c->fall, M2 * 4)) ||
        (rc = ensure(c, c->mstat, M2 * 8)) || (rc = ensure(c, c->pidx, (size_t)M * 4)) ||
        (rc = ensure(c, c->heavy, (size_t)M * 4)) ||
        (rc = ensure(c, c->mlist, (size_t)M * 4)) || (rc = ensure(c, c->mcnt, (size_t)M * 8)) ||
        (rc = ensure(c, c->moff, (size_t)M * 8)) || (rc = ensure(c, c->minfo, (size_t)M * 16)) ||
        (rc = ensure(c, c->mreg, (size_t)M * 8)) || (rc = ensure(c, c->icnt, (size_t)M * 4)) ||
        (rc = ensure(c, c->ioff, (size_t)M * 4)) ||
        (rc = ensure_scan(c, std::max<uint64_t>(std::max<uint64_t>(M2, (uint64_t)C / 32 + 2), (uint64_t)NC + 1))))
        return rc;
    if ((rc = ensure_events(c))) return rc;
    reset_stats_host(c);
    if (!c->stats_zero)                              // else the last tick's reset pass zeroed them
        HIPCHK(hipMemcpyAsync(c->stats, c->hstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
    c->stats_zero = false;
    DevStats* st = c->stats;

    TickBufs b{};
    b.w = world(c);
    b.ops = ops; b.m = M; b.stamp_base = c->stamp_base;
    b.mbit = c->mpar ? MOVER_B : MOVER_A;
    b.mstale = c->mpar ? MOVER_A : MOVER_B;
    b.ol_tag = 0;
    if (c->wd.ol_pre) {                               // the world's routing deduped its ops already
        const uint32_t k = c->wd.ol_pre;
        c->wd.ol_pre = 0;
        const OpSeg& s0 = c->segs[0];
        if (!s0.host && !s0.rows && s0.dev == c->wd.ops && s0.n == k) {
            b.op0 = k;                                // same session: its dedupe words are this tick's
            b.ol_tag = c->wd.kept_tag;
        }
    }
    if (!b.ol_tag && (rc = next_ol_tag(c, &b.ol_tag))) return rc;
    b.stamps = stamps;
    b.diff_u = c->diff_u;
    b.compact = c->mover_compact;
    b.heavy = P<uint32_t>(c->heavy);
    // heavy-first only for few movers (a world strip): the tick's tail is then
    // the longest walk; with many movers the one-wave-per-mover dispatch balances
    b.heavy_min = (b.compact && M <= c->heavy_maxm) ? c->heavy_min : 0u;
    b.walk_min = c->walk_min;
    b.rank_sort = c->rank_sort;
    b.grid_cap = c->grid_cap;
    b.pair_max = c->pair_auto ? (c->cand_mean <= gw_ctx::PAIR_MEAN ? gw_ctx::PAIR_AUTO : 0u) : c->pair_max;
    // dirty-cell span by cell count: a world strip's few cells spread over
    // more waves (1M world at 8 strips, 57k cells: grid 37 -> 30 us at 2)
    // (above 2M cells 64: config #4's 4.4M cells grid 270 -> 260 us, config #5's
    // 6.9M 513 -> 484 us)
    b.dirty_span = c->dirty_span ? c->dirty_span
                                 : (NC > (1u << 21) ? 64u : NC > (1u << 20) ? 16u : NC > (1u << 17) ? 8u : 2u);
    // decomposed world of >= 2 strips: long movers (a one-strip world holds every pair)
    b.long_step = (c->wd.on && c->wd.g.ranks > 1) ? c->wd.g.max_step : INFINITY;
    b.longs = c->wd.tick_longs;                      // the long lists queued for this tick (world.cpp)
    b.n_long = c->wd.tick_nlong;
    b.conflicts = c->wd.on ? &st->n_conflicts : nullptr;   // per attempt: a redo must not count twice
    // (the multi-gate collect; GW_GATE_COUNTS=0: its count pass walks every window, A/B)
    static const bool gcounts_on = !getenv("GW_GATE_COUNTS") || atoi(getenv("GW_GATE_COUNTS")) != 0;
    b.gate_counts = (gcounts_on && c->max_gate + 1u > 2u && c->max_gate + 1u <= GATE_DIRECT_MAX) ? c->max_gate + 1u : 0u;
    c->wd.tick_longs = nullptr;
    c->wd.tick_nlong = 0;
    b.ol = c->ol;
    b.st = st;
    b.gn_nxt = c->gnb[c->gcur ^ 1]; b.start_nxt = c->gsb[c->gcur ^ 1];
    b.dep = c->dep; b.arr = c->arr; b.cnt_new = c->cnt_new;
    b.gm_cnt = c->gm_cnt; b.gm_start = c->gm_start; b.gm = P<MEnt>(c->gm);
    b.mtmp = P<MEnt>(c->mtmp); b.mcell = P<uint4>(c->mcell);
    b.cand = P<uint64_t>(c->cand); b.reg = P<uint64_t>(c->reg); b.pidx = P<uint32_t>(c->pidx);
    b.ownc = P<unsigned long long>(c->ownc); b.mirc = P<unsigned long long>(c->mirc);
    b.big = P<uint32_t>(c->big);
    b.fall = P<uint32_t>(c->fall);
    b.half_rows = c->half_rows;
    b.gate_lane_max = c->gate_lane_max;
    b.bk_flat = c->bk_flat;
    b.post_split = c->post_split;
    b.place_split = c->place_split;
    b.mstat = P<unsigned long long>(c->mstat);
    b.movbit = c->movbit; b.gmi = c->gmi;
    b.mlist = P<uint32_t>(c->mlist);
    b.mcnt = P<unsigned long long>(c->mcnt); b.moff = P<unsigned long long>(c->moff);
    b.minfo = P<uint4>(c->minfo); b.mreg = P<unsigned long long>(c->mreg);
    b.icnt = P<uint32_t>(c->icnt); b.ioff = P<uint32_t>(c->ioff);
    b.wbits = ceil_log2(C);
    small_mode(c, b);
    if (b.small_ents || b.pair_max || !ev_on) {
        b.rowrec = nullptr;                          // only k_mover reads the row ranges
    } else {
        if ((rc = ensure(c, c->rowrec, M2 * RR_ROWS * 16))) return rc;
        b.rowrec = P<uint4>(c->rowrec);
    }
    bind_events(c, b);
    if (!c->ev_est) c->ev_est = 16ull * M;
    choose_buckets(c, b);
    if (c->bk_split_w != b.wbits) {                  // slot bits changed: uniform bounds until a tick's quantiles
        launch_bk_split_init(b.bk_split, b.wbits, c->st);
        c->bk_split_w = b.wbits;
    }

    prof_begin(c, "ops");
    c->cells_zero = false;                           // counters are in flight until the grid stage ends
    tick_ops(b, c->st);
    prof_end(c, (uint64_t)M * 24);
    prof_begin(c, "grid");
    // with events, the dirty cells are merged in the bounds' launch (GW_DIRTY_SPLIT=1: their own)
    const bool dirty_later = ev_on && !c->dirty_split;
    tick_grid(b, c->sc, c->st, !dirty_later);
    HIPCHK(hipEventRecord(c->ev_grid, c->st));        // a following collect's flag compaction may start here
    c->mpar ^= 1u;                                   // the next rebuild drops this tick's mover bits
    c->cells_zero = true;
    size_t s_grid = prof_end(c, 0);
    c->gcur ^= 1;                                    // the new grid is current from here on
    const TickBufs bg = b;                           // (the buffers before the flip)
    b.w = world(c);
    prof_begin(c, "movers");
    if (ev_on) tick_movers(b, c->sc, c->st, dirty_later ? &bg : nullptr);
    size_t s_movers = prof_end(c, 0);
    prof_begin(c, "diff");
    if (ev_on) tick_diff(b, c->st);
    size_t s_diff = prof_end(c, 0);
    HIPCHK(hipEventRecord(c->ev_diff, c->st));        // a following collect may start here (st2)
    prof_begin(c, "events");
    if (ev_on) tick_events(b, c->sc, c->st);
    size_t s_events = prof_end(c, 0);
    HIPCHK(hipGetLastError());
    c->segs.clear();
    c->pend_host.clear();
    c->stamp_base += M;
    auto& p = c->pt;
    p.on = true;
    p.copied = false;
    p.M = M; p.C = C; p.NC = NC; p.flags = flags;
    p.s_grid = s_grid; p.s_movers = s_movers; p.s_diff = s_diff; p.s_events = s_events;
    p.b = b;
    if ((flags & GW_TICK_DEFER) && !(flags & GW_TICK_COPY_TO_HOST) && !host_ops) {
        // no host sync now: the next call that needs the results settles it
        // (a collect reads the statistics with its own; anything else copies them)
        p.copied = false;
        out->ops = M;
        return 0;
    }
    return finish_tick(c, out);
}

int gw_sync_collect(gw_ctx* c, uint32_t flags, gw_sync_out* out) {
    if (!c || !out) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    memset(out, 0, sizeof *out);
    const uint32_t C = c->total_slots;
    int rc;
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    const uint32_t G = (uint32_t)c->max_gate + 1;
    c->gate_off.assign((size_t)G + 1, 0);
    if (C == 0) {
        out->gate_off = c->gate_off.data();
        out->n_gates = G;
        return 0;
    }
    if (c->grid_dirty && (rc = settle(c))) return rc;
    if ((rc = rebuild_grid(c))) return rc;
    DevStats* st = c->cstats;                        // its overflow flag is zeroed by the compaction
    if ((rc = ensure(c, c->fbits, (size_t)C * 4)) || (rc = ensure(c, c->flagged, (size_t)C * 4)) ||
        (rc = ensure(c, c->rec_cnt, (size_t)C * 4)) || (rc = ensure(c, c->rec_off, (size_t)C * 8)) ||
        (rc = ensure_scan(c, C)))
        return rc;
    // records land in a buffer sized from the last collect; if it was too
    // small, the write pass (which reads only the compacted list) reruns
    c->rec_cap = std::max<uint64_t>(c->rec_cap, 4ull * C + 1024);
    if ((rc = ensure(c, c->rec0, c->rec_cap * sizeof(gw_sync_record)))) return rc;
    const World w = world(c);
    // only slots with an op or a restore since the last collect can be flagged:
    // the passes over the flagged list are sized by that bound, not the slots
    const uint32_t NFM = (uint32_t)std::min<uint64_t>(C, std::max<uint64_t>(c->flag_bound, 1));
    c->flag_bound = 0;
    // small-space mode: every space's grid fits in LDS (config #4's many small spaces)
    uint32_t max_ents = 0, max_cells = 0;
    for (auto& sp : c->spaces)
        if (sp.alive) {
            max_ents = std::max(max_ents, sp.cap);
            max_cells = std::max(max_cells, (uint32_t)(sp.p.W * sp.p.H));
        }
    const uint32_t n_sp = (uint32_t)c->spaces.size();
    static const bool small_on = !getenv("GW_SMALL") || atoi(getenv("GW_SMALL")) != 0;
    const bool small = small_on && n_sp >= 2 &&
                       (size_t)max_ents * sizeof(GEnt) + ((size_t)max_cells + 1) * 4 <= SMALL_LDS_MAX;
    // the spaces' runs of the flagged list: zeroed by the compaction, set by the count pass
    if (small && (rc = ensure(c, c->srange, (size_t)n_sp * 8))) return rc;
    uint32_t* sfirst = small ? P<uint32_t>(c->srange) : nullptr;
    uint32_t* slast = small ? sfirst + n_sp : nullptr;
    // after a deferred tick the flag, count and write passes need only its
    // diff (the new grid, states and cached neighbour counts), not its events
    // stage: they run on st2 beside it, and st waits for them before the
    // statistics publish (per-stage profiling keeps one stream)
    const bool ovl = c->overlap && c->pt.on && !c->pt.copied && c->pt.M >= c->overlap_min && c->prof != 1;
    const bool by_client = (flags & GW_SYNC_BY_CLIENT) != 0;
    // several gate ids in use: records straight into their gates' partitions
    // (counts and offsets per (gate, entry), gate-major; sync.hip)
    static const bool gdirect_on = !getenv("GW_GATE_DIRECT") || atoi(getenv("GW_GATE_DIRECT")) != 0;
    const bool gdirect = gdirect_on && G > 2 && G <= GATE_DIRECT_MAX && !by_client && !small;
    const uint64_t NG = gdirect ? (uint64_t)G * NFM : NFM;   // count / offset entries
    if (gdirect && ((rc = ensure(c, c->rec_cnt, NG * 4)) || (rc = ensure(c, c->rec_off, NG * 8)) ||
                    (rc = ensure_scan(c, NG))))
        return rc;
    hipStream_t cs = c->st;
    ScanCtx* csc = &c->sc;
    if (ovl) {
        if ((rc = ensure_scan2(c, std::max<uint64_t>(C, NG), c->st2))) return rc;
        HIPCHK(hipStreamWaitEvent(c->st2, c->ev_grid, 0));   // the flags are final after the grid stage
        cs = c->st2;
        csc = &c->sc2;
    }
    prof_begin(c, "sync_flagged");
    launch_flag_compact(c->flags, C, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), *csc, &st->flagged,
                        &st->overflow, sfirst, small ? 2 * n_sp : 0u, cs);
    prof_end(c, (uint64_t)C * 4 * 2);
    if (ovl) HIPCHK(hipStreamWaitEvent(c->st2, c->ev_diff, 0));   // the counts read the diff's cache
    const uint64_t* nf = (const uint64_t*)&st->flagged;
    prof_begin(c, "sync_count");
    if (gdirect) {
        launch_sync_gates(w, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), nf, NFM, G, P<uint32_t>(c->rec_cnt), cs);
        scan_u32_u64(P<uint32_t>(c->rec_cnt), P<uint64_t>(c->rec_off), NG, nullptr, *csc,
                     (uint64_t*)&st->rec_total, cs);
    } else {
        launch_sync_count(w, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), nf, NFM, P<uint32_t>(c->rec_cnt), sfirst,
                          slast, cs);
        scan_u32_u64(P<uint32_t>(c->rec_cnt), P<uint64_t>(c->rec_off), NFM, nf, *csc,
                     (uint64_t*)&st->rec_total, cs);
    }
    size_t s_count = prof_end(c, 0);
    // per-client grouping (GW_SYNC_BY_CLIENT): the write pass leaves (watcher,
    // entity) pairs, the sort's keys and values; the records are built once
    // after the sort (not written, keyed, sorted and gathered at 24 B)
    const bool pairs = by_client && !small;
    if (pairs && ((rc = ensure(c, c->gk0, c->rec_cap * 8)) || (rc = ensure(c, c->pay, (size_t)NFM * 16))))
        return rc;
    prof_begin(c, "sync_write");
    // short lists two per wave when the last collect averaged <= 64 records per
    // flagged entity (config #5: write 1081 -> 852 us; config #3's 146: +4 us)
    const bool sw_halves = c->sw_halves < 0 ? c->rec_per_flagged <= 64.0 : c->sw_halves > 0;
    auto write_pass = [&](hipStream_t ws) {
        if (gdirect)
            launch_sync_write_gates(w, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), nf, NFM, G,
                                    P<uint64_t>(c->rec_off), P<gw_sync_record>(c->rec0), c->rec_cap, st, ws);
        else if (small)
            launch_sync_write_small(w, n_sp, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), P<uint64_t>(c->rec_off),
                                    P<uint32_t>(c->rec_cnt), P<gw_sync_record>(c->rec0), c->rec_cap, st,
                                    sfirst, slast, max_ents, max_cells, ws);
        else
            launch_sync_write(w, P<uint32_t>(c->flagged), P<uint32_t>(c->fbits), nf, NFM, P<uint64_t>(c->rec_off),
                              P<uint32_t>(c->rec_cnt), P<gw_sync_record>(c->rec0), c->rec_cap, st, ws,
                              pairs ? P<uint64_t>(c->gk0) : nullptr, pairs ? P<float4>(c->pay) : nullptr,
                              sw_halves);
    };
    write_pass(cs);
    size_t s_write = prof_end(c, 0);
    HIPCHK(hipGetLastError());
    if (ovl) {                                           // the publish waits for the collect's passes
        HIPCHK(hipEventRecord(c->ev_col, c->st2));
        HIPCHK(hipStreamWaitEvent(c->st, c->ev_col, 0));
    }
    if ((rc = read_cstats(c))) return rc;                // the one host sync
    if ((rc = settle(c))) return rc;                     // a deferred tick: its stats came with it
    const uint64_t R = c->hcstats->rec_total;
    const uint64_t NF = c->hcstats->flagged;
    if (NF) c->rec_per_flagged = (double)R / (double)NF;
    if (c->hcstats->overflow) {
        c->rec_cap = R + R / 4 + 1024;
        if ((rc = ensure(c, c->rec0, c->rec_cap * sizeof(gw_sync_record)))) return rc;
        if (pairs && (rc = ensure(c, c->gk0, c->rec_cap * 8))) return rc;
        c->hcstats->overflow = 0;
        HIPCHK(hipMemcpyAsync(c->cstats, c->hcstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
        write_pass(c->st);
        HIPCHK(hipGetLastError());
        if ((rc = read_cstats(c))) return rc;
        if (c->hcstats->overflow) return set_err(c, GW_ENOMEM, "sync record buffer overflowed twice");
    }
    gw_sync_record* recs = P<gw_sync_record>(c->rec0);
    bool gates_done = false;
    if (gdirect) {                                       // the partitions' first records came with the sync
        for (uint32_t g = 0; g < G; ++g) c->gate_off[g] = c->hcstats->gate_base[g];
        c->gate_off[G] = R;
        gates_done = true;
    }
    if (pairs) {
        // (watcher, flagged index) pairs, packed u64, in entity order -> stable
        // sort by watcher -> with several gates in use a stable sort of the
        // pairs' gates -> records and client table: order (gate, watcher, entity)
        prof_begin(c, "sync_clients");
        gates_done = true;
        const uint32_t* idx = nullptr;
        uint64_t* wp = P<uint64_t>(c->gk0);
        for (uint32_t g = 0; g <= G; ++g) c->gate_off[g] = (g == G) ? R : 0;   // one gate id in use
        if (R) {
            if ((rc = ensure(c, c->gk1, R * 8))) return rc;
            RadixTmp rt;
            if ((rc = radix_tmp(c, R, rt))) return rc;
            if (R > 1 && sort_pairs64(P<uint64_t>(c->gk0), P<uint64_t>(c->gk1), R, nullptr, 0, ceil_log2(C), rt, c->st))
                wp = P<uint64_t>(c->gk1);
            if (G > 2) {
                if ((rc = ensure(c, c->gv0, R * 4)) || (rc = ensure(c, c->gv1, R * 4)) ||
                    (rc = ensure(c, c->m_flag, R * 4)) || (rc = ensure(c, c->m_at, R * 4)) ||
                    (rc = ensure(c, c->gate_hist, (size_t)65536 * 4)))
                    return rc;
                uint32_t *ka = P<uint32_t>(c->gv0), *va = P<uint32_t>(c->gv1);
                HIPCHK(hipMemsetAsync(c->gate_hist.p, 0, (size_t)G * 4, c->st));
                launch_gate_keys(wp, c->gate, R, ka, va, P<uint32_t>(c->gate_hist), c->st);
                std::vector<uint32_t> h(G);
                HIPCHK(hipMemcpyAsync(h.data(), c->gate_hist.p, (size_t)G * 4, hipMemcpyDeviceToHost, c->st));
                HIPCHK(hipStreamSynchronize(c->st));
                uint32_t nonzero = 0;
                uint64_t acc = 0;
                for (uint32_t g = 0; g < G; ++g) { nonzero += h[g] != 0; c->gate_off[g] = acc; acc += h[g]; }
                c->gate_off[G] = acc;
                if (nonzero > 1) {
                    const int gs = sort_u32_u32(ka, va, P<uint32_t>(c->m_flag), P<uint32_t>(c->m_at), R, nullptr, 0,
                                                ceil_log2(G), rt, c->st);
                    idx = gs ? P<uint32_t>(c->m_at) : va;
                }
            }
            if ((rc = ensure(c, c->cl_slot, R * 4)) || (rc = ensure(c, c->cl_off, (R + 1) * 8)) ||
                (rc = ensure_scan(c, R)))
                return rc;
            launch_records_seg(w, wp, idx, P<uint32_t>(c->flagged), P<float4>(c->pay), R, recs,
                               P<uint32_t>(c->cl_slot), P<uint64_t>(c->cl_off), c->scal32 + 1, c->sc, c->st);
            HIPCHK(hipGetLastError());
        }
        prof_end(c, R * (8 * 2 * 3 + 24));
    }
    // ---- per-client grouping: stable sort by watcher (the gate grouping below
    // is stable too, so the order becomes (gate, watcher, entity)) ---------
    if (by_client && !pairs && R > 1) {
        prof_begin(c, "sync_clients");
        if ((rc = ensure(c, c->gk0, R * 4)) || (rc = ensure(c, c->gv0, R * 4)) || (rc = ensure(c, c->gk1, R * 4)) ||
            (rc = ensure(c, c->gv1, R * 4)) || (rc = ensure(c, c->rec1, R * sizeof(gw_sync_record))))
            return rc;
        RadixTmp rt;
        if ((rc = radix_tmp(c, R, rt))) return rc;
        launch_watcher_keys(recs, R, P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), c->st);
        const int wsel = sort_u32_u32(P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), P<uint32_t>(c->gk1),
                                      P<uint32_t>(c->gv1), R, nullptr, 0, ceil_log2(C), rt, c->st);
        launch_gather_records(recs, wsel ? P<uint32_t>(c->gv1) : P<uint32_t>(c->gv0), nullptr, R,
                              P<gw_sync_record>(c->rec1), c->st);
        std::swap(c->rec0, c->rec1);
        recs = P<gw_sync_record>(c->rec0);
        prof_end(c, R * (24 * 2 + 8 * 4));
    }
    // ---- per-gate grouping (stable, keeps the entity order) -------------
    if (gates_done) {
    } else if (R && G > 2) {
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
    uint32_t n_clients = 0;
    if (by_client && R) {
        if (!pairs) {                                 // (the pairs path built the table with its records)
            if ((rc = ensure(c, c->gk0, R * 4)) || (rc = ensure(c, c->gk1, R * 4)) ||
                (rc = ensure(c, c->cl_slot, R * 4)) || (rc = ensure(c, c->cl_off, (R + 1) * 8)) ||
                (rc = ensure_scan(c, R)))
                return rc;
            launch_client_segments(recs, R, P<uint32_t>(c->gk0), P<uint32_t>(c->gk1), c->scal32 + 1,
                                   P<uint32_t>(c->cl_slot), P<uint64_t>(c->cl_off), c->sc, c->st);
        }
        HIPCHK(hipMemcpyAsync(&n_clients, c->scal32 + 1, 4, hipMemcpyDeviceToHost, c->st));
    }
    // the stream is synced again only for host outputs (records, client
    // table): without them the caller may queue the next tick behind the
    // collect's tail at once, and device_us stays 0 (as for gw_tick)
    if ((flags & GW_SYNC_COPY_TO_HOST) || by_client) {
        HIPCHK(hipEventRecord(c->ev_t1, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1);
        out->device_us = ms * 1000.0;
    }
    out->n_rec = R;
    if (by_client) {
        out->n_clients = n_clients;
        out->client_slot_dev = P<uint32_t>(c->cl_slot);
        out->client_off_dev = P<uint64_t>(c->cl_off);
        if (flags & GW_SYNC_COPY_TO_HOST) {
            if ((rc = ensure_host(c, c->h_cl_slot, (size_t)std::max<uint32_t>(n_clients, 1) * 4)) ||
                (rc = ensure_host(c, c->h_cl_off, ((size_t)n_clients + 1) * 8)))
                return rc;
            if (n_clients) {
                HIPCHK(hipMemcpyAsync(c->h_cl_slot.p, c->cl_slot.p, (size_t)n_clients * 4, hipMemcpyDeviceToHost, c->st));
                HIPCHK(hipMemcpyAsync(c->h_cl_off.p, c->cl_off.p, ((size_t)n_clients + 1) * 8, hipMemcpyDeviceToHost, c->st));
                HIPCHK(hipStreamSynchronize(c->st));
            } else {
                *(uint64_t*)c->h_cl_off.p = 0;
            }
            out->client_slot = (const uint32_t*)c->h_cl_slot.p;
            out->client_off = (const uint64_t*)c->h_cl_off.p;
        }
    }
    out->flagged = NF;
    out->rec_dev = recs;
    c->last_rec = recs;
    c->last_R = R;
    out->gate_off = c->gate_off.data();
    out->n_gates = G;
    out->bytes_alg = 24ull * R;
    if (c->prof) {
        prof_set_bytes(c, s_count, NF * 32);
        prof_set_bytes(c, s_write, 24ull * R + NF * 32);
    }
    if (flags & GW_SYNC_COPY_TO_HOST) {
        if ((rc = ensure_host(c, c->h_rec, std::max<uint64_t>(R, 1) * sizeof(gw_sync_record)))) return rc;
        if (R) HIPCHK(hipMemcpyAsync(c->h_rec.p, recs, R * sizeof(gw_sync_record), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        out->rec = (const gw_sync_record*)c->h_rec.p;
    }
    return 0;
}

// ---- client messages -------------------------------
// Stable grouping of R records of `words` u32 in m.a (first word = watcher):
// by watcher first (by_watcher), then by gate(watcher); m.goff = gate offsets.
static int group_msgs(gw_ctx* c, gw_ctx::MsgBufs& m, uint64_t R, int words, bool by_watcher) {
    const uint32_t G = (uint32_t)c->max_gate + 1;
    m.goff.assign((size_t)G + 1, 0);
    if (!R) return 0;
    int rc;
    if ((rc = ensure(c, c->gk0, R * 4)) || (rc = ensure(c, c->gv0, R * 4)) || (rc = ensure(c, c->gk1, R * 4)) ||
        (rc = ensure(c, c->gv1, R * 4)) || (rc = ensure(c, m.b, R * words * 4)))
        return rc;
    RadixTmp rt;
    if ((rc = radix_tmp(c, R, rt))) return rc;
    auto sort_by = [&](const uint16_t* gate, int bits) {
        launch_msg_keys(P<uint32_t>(m.a), words, R, gate, P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), c->st);
        const int sel = sort_u32_u32(P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), P<uint32_t>(c->gk1),
                                     P<uint32_t>(c->gv1), R, nullptr, 0, bits, rt, c->st);
        launch_msg_gather(P<uint32_t>(m.a), words, sel ? P<uint32_t>(c->gv1) : P<uint32_t>(c->gv0), R,
                          P<uint32_t>(m.b), c->st);
        std::swap(m.a, m.b);
    };
    if (by_watcher && R > 1) sort_by(nullptr, ceil_log2(c->total_slots));
    if (G > 2) {
        if ((rc = ensure(c, c->gate_hist, (size_t)65536 * 4))) return rc;
        HIPCHK(hipMemsetAsync(c->gate_hist.p, 0, (size_t)G * 4, c->st));
        launch_msg_gate_hist(P<uint32_t>(m.a), words, R, c->gate, P<uint32_t>(c->gate_hist), c->st);
        std::vector<uint32_t> h(G);
        HIPCHK(hipMemcpyAsync(h.data(), c->gate_hist.p, (size_t)G * 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        uint32_t nonzero = 0;
        uint64_t acc = 0;
        for (uint32_t g = 0; g < G; ++g) { nonzero += h[g] != 0; m.goff[g] = acc; acc += h[g]; }
        m.goff[G] = acc;
        if (nonzero > 1) sort_by(c->gate, ceil_log2(G));
    } else {
        for (uint32_t g = 0; g <= G; ++g) m.goff[g] = (g == G) ? R : 0;   // one gate id in use
    }
    return 0;
}

static int msg_out(gw_ctx* c, gw_ctx::MsgBufs& m, uint64_t R, int words, uint32_t flags, gw_msg_out* o) {
    o->rec_dev = m.a.p;
    o->n_rec = R;
    o->gate_off = m.goff.data();
    o->n_gates = (uint32_t)m.goff.size() - 1;
    o->bytes_alg = R * words * 4;
    if (flags & GW_MSG_COPY_TO_HOST) {
        int rc;
        if ((rc = ensure_host(c, m.h, std::max<uint64_t>(R, 1) * words * 4))) return rc;
        if (R) HIPCHK(hipMemcpyAsync(m.h.p, m.a.p, R * words * 4, hipMemcpyDeviceToHost, c->st));
        o->rec = m.h.p;
    }
    return 0;
}

int gw_client_events(gw_ctx* c, uint32_t flags, gw_msg_out* create, gw_msg_out* destroy) {
    if (!c || !create || !destroy) return GW_EINVAL;
    int rc;
    if ((rc = settle(c))) return rc;
    (void)hipSetDevice(c->dev);
    memset(create, 0, sizeof *create);
    memset(destroy, 0, sizeof *destroy);
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    const gw_tick_out& t = c->last_out;
    const gw_event* evs[2] = {t.enter_dev, t.leave_dev};
    const uint64_t ns[2] = {evs[0] ? t.n_enter : 0, evs[1] ? t.n_leave : 0};
    gw_ctx::MsgBufs* ms[2] = {&c->m_create, &c->m_destroy};
    gw_msg_out* outs[2] = {create, destroy};
    // both kinds' messages (one look-back pass each), then one host sync for
    // both counts
    uint32_t Rk[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
        const uint64_t n = ns[k];
        if (!n) continue;
        if (n >= 0xffffffffull) return set_err(c, GW_ERANGE, "too many events (%llu)", (unsigned long long)n);
        if ((rc = ensure_scan(c, n)) || (rc = ensure(c, ms[k]->a, n * (k == 0 ? 6 : 2) * 4))) return rc;
        launch_event_client_compact(evs[k], n, c->gate, c->rec, P<uint32_t>(ms[k]->a), k == 0, c->scal32 + 2 + k,
                                    c->sc, c->st);
    }
    if (ns[0] || ns[1]) {
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(Rk, c->scal32 + 2, 8, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        for (int k = 0; k < 2; ++k)
            if (!ns[k]) Rk[k] = 0;
    }
    for (int k = 0; k < 2; ++k) {
        const int words = k == 0 ? 6 : 2;
        if ((rc = group_msgs(c, *ms[k], Rk[k], words, false)) || (rc = msg_out(c, *ms[k], Rk[k], words, flags, outs[k])))
            return rc;
        outs[k]->bytes_alg += ns[k] * 8;
    }
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    float ms_ = 0;
    (void)hipEventElapsedTime(&ms_, c->ev_t0, c->ev_t1);
    create->device_us = destroy->device_us = ms_ * 1000.0;
    return 0;
}

int gw_fanout(gw_ctx* c, const uint32_t* slots, uint32_t n, uint32_t flags, gw_msg_out* out) {
    if (!c || !out || (n && !slots)) return GW_EINVAL;
    int rc;
    if ((rc = settle(c))) return rc;
    (void)hipSetDevice(c->dev);
    memset(out, 0, sizeof *out);
    // the calls are checked while they are staged in pinned memory (an async
    // copy from there instead of a pageable one)
    if (n && (rc = ensure_host(c, c->h_items, (size_t)n * 4))) return rc;
    uint32_t* hi = (uint32_t*)c->h_items.p;
    uint32_t bad = 0;
    const uint32_t C = c->total_slots;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t s = slots[k];
        bad |= s >= C;
        hi[k] = s;
    }
    if (bad)
        for (uint32_t k = 0; k < n; ++k)
            if (slots[k] >= C) return set_err(c, GW_ERANGE, "fanout: slot %u out of range", slots[k]);
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    gw_ctx::MsgBufs& m = c->m_fanout;
    const uint32_t G = (uint32_t)c->max_gate + 1;
    m.goff.assign((size_t)G + 1, 0);
    uint64_t R = 0;
    if (n) {
        if ((rc = rebuild_grid(c))) return rc;
        if ((rc = ensure(c, c->m_items, (size_t)n * 4)) || (rc = ensure(c, c->m_cnt, (size_t)n * 4)) ||
            (rc = ensure(c, c->m_off, ((size_t)n + 1) * 8)) || (rc = ensure_scan(c, n)))
            return rc;
        HIPCHK(hipMemcpyAsync(c->m_items.p, hi, (size_t)n * 4, hipMemcpyHostToDevice, c->st));
        const World w = world(c);
        launch_fanout(w, P<uint32_t>(c->m_items), n, P<uint32_t>(c->m_cnt), nullptr, nullptr, c->st);
        uint64_t* tot = P<uint64_t>(c->m_off) + n;   // the total lands after the offsets
        scan_u32_u64(P<uint32_t>(c->m_cnt), P<uint64_t>(c->m_off), n, nullptr, c->sc, tot, c->st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&R, tot, 8, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
    }
    if (R) {
        // deliveries as packed (watcher, item) pairs, a stable radix sort by
        // watcher (item order inside each watcher), then, with several gates in
        // use, a stable sort of the pairs' gates; the 12-B records are written once
        if ((rc = ensure(c, c->gk0, R * 8)) || (rc = ensure(c, c->gk1, R * 8)) ||
            (rc = ensure(c, m.a, R * sizeof(gw_fanout_rec))))
            return rc;
        RadixTmp rt;
        if ((rc = radix_tmp(c, R, rt))) return rc;
        const World w = world(c);
        launch_fanout(w, P<uint32_t>(c->m_items), n, nullptr, P<uint64_t>(c->m_off), P<uint64_t>(c->gk0), c->st);
        uint64_t* wp = P<uint64_t>(c->gk0);
        if (sort_pairs64(P<uint64_t>(c->gk0), P<uint64_t>(c->gk1), R, nullptr, 0, ceil_log2(c->total_slots), rt,
                         c->st))
            wp = P<uint64_t>(c->gk1);
        const uint32_t* idx = nullptr;
        if (G > 2) {
            if ((rc = ensure(c, c->gv0, R * 4)) || (rc = ensure(c, c->gv1, R * 4)) ||
                (rc = ensure(c, c->m_flag, R * 4)) || (rc = ensure(c, c->m_at, R * 4)) ||
                (rc = ensure(c, c->gate_hist, (size_t)65536 * 4)))
                return rc;
            uint32_t *ka = P<uint32_t>(c->gv0), *va = P<uint32_t>(c->gv1);
            HIPCHK(hipMemsetAsync(c->gate_hist.p, 0, (size_t)G * 4, c->st));
            launch_gate_keys(wp, c->gate, R, ka, va, P<uint32_t>(c->gate_hist), c->st);
            std::vector<uint32_t> h(G);
            HIPCHK(hipMemcpyAsync(h.data(), c->gate_hist.p, (size_t)G * 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
            uint32_t nonzero = 0;
            uint64_t acc = 0;
            for (uint32_t g = 0; g < G; ++g) { nonzero += h[g] != 0; m.goff[g] = acc; acc += h[g]; }
            m.goff[G] = acc;
            if (nonzero > 1) {
                const int gs = sort_u32_u32(ka, va, P<uint32_t>(c->m_flag), P<uint32_t>(c->m_at), R, nullptr, 0,
                                            ceil_log2(G), rt, c->st);
                idx = gs ? P<uint32_t>(c->m_at) : va;
            }
        } else {
            for (uint32_t g = 0; g <= G; ++g) m.goff[g] = (g == G) ? R : 0;   // one gate id in use
        }
        launch_fanout_final(wp, idx, P<uint32_t>(c->m_items), R, P<gw_fanout_rec>(m.a), c->st);
        HIPCHK(hipGetLastError());
    }
    if ((rc = msg_out(c, m, R, 3, flags, out))) return rc;
    out->bytes_alg += (uint64_t)n * 4;
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    float ms_ = 0;
    (void)hipEventElapsedTime(&ms_, c->ev_t0, c->ev_t1);
    out->device_us = ms_ * 1000.0;
    return 0;
}

int gw_neighbors(gw_ctx* c, uint32_t slot, uint32_t* buf, uint32_t cap, uint32_t* n) {
    if (!c || !n) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    if (slot >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slot);
    int rc;
    if ((rc = rebuild_grid(c))) return rc;
    const uint32_t qcap = c->total_slots;
    if ((rc = ensure(c, c->qbuf, ((size_t)qcap + 1) * 4))) return rc;
    uint32_t* q = P<uint32_t>(c->qbuf);
    launch_neighbors(world(c), slot, q + 1, q, qcap, c->st);
    HIPCHK(hipGetLastError());
    uint32_t cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, q, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    std::vector<uint32_t> v(std::min(cnt, qcap));
    if (!v.empty()) HIPCHK(hipMemcpyAsync(v.data(), q + 1, v.size() * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    std::sort(v.begin(), v.end());
    *n = cnt;
    uint32_t k = std::min<uint32_t>((uint32_t)v.size(), cap);
    if (buf && k) memcpy(buf, v.data(), (size_t)k * 4);
    return 0;
}

int gw_total_neighbors(gw_ctx* c, uint64_t* out) {
    if (!c || !out) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    *out = 0;
    if (!c->total_slots) return 0;
    int rc;
    if ((rc = rebuild_grid(c))) return rc;
    HIPCHK(hipMemsetAsync(c->scal32, 0, 8, c->st));
    launch_count_all(world(c), c->h_present, (unsigned long long*)c->scal32, c->st);
    HIPCHK(hipGetLastError());
    unsigned long long t = 0;
    HIPCHK(hipMemcpyAsync(&t, c->scal32, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    *out = t;
    return 0;
}

int gw_set_profiling(gw_ctx* c, int enable) {
    if (!c) return GW_EINVAL;
    c->prof = enable < 0 ? 0 : (enable > 2 ? 1 : enable);
    return 0;
}

int gw_get_stage_times(gw_ctx* c, gw_stage_times* out) {
    if (!c || !out) return GW_EINVAL;
    prof_collect(c);                 // waits for the last recorded stage, then clears the record
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
int gw_step(gw_ctx* c, const gw_op* ops, uint32_t n, int ops_on_device, uint32_t tick_flags, uint32_t sync_flags,
            gw_tick_out* tick_out, gw_sync_out* sync_out) {
    if (!c || !tick_out || !sync_out) return GW_EINVAL;
    int rc;
    if (c->wd.on)                                    // a world strip: route + exchange + queue (even with no ops)
        rc = ops_on_device ? gw_world_step(c, ops, n) : gw_world_step_host(c, ops, n);
    else
        rc = n ? (ops_on_device ? gw_submit_device(c, ops, n) : gw_submit(c, ops, n)) : 0;
    if (rc) return rc;
    const uint32_t tf = tick_flags | ((ops_on_device && !(tick_flags & GW_TICK_COPY_TO_HOST)) ? GW_TICK_DEFER : 0u);
    if ((rc = gw_tick(c, tf, tick_out))) return rc;
    if ((rc = gw_sync_collect(c, sync_flags, sync_out))) return rc;
    return (tf & GW_TICK_DEFER) ? gw_tick_result(c, tick_out) : 0;
}

int gw_replay(gw_ctx* c, const gw_op* dev_ops, uint32_t n, uint64_t stride_ops, uint32_t ticks, uint32_t sync_flags,
              gw_replay_sum* sum) {
    if (!c || !sum || (n && !dev_ops)) return GW_EINVAL;
    memset(sum, 0, sizeof *sum);
    for (uint32_t t = 0; t < ticks; ++t) {
        gw_tick_out to;
        gw_sync_out so;
        if (int rc = gw_step(c, dev_ops + (size_t)t * stride_ops, n, 1, 0, sync_flags, &to, &so)) return rc;
        sum->ops += to.ops;
        sum->movers += to.movers;
        sum->n_enter += to.n_enter;
        sum->n_leave += to.n_leave;
        sum->n_rec += so.n_rec;
        sum->pairs_tested += to.pairs_tested;
        sum->nbr_old += to.nbr_old;
        sum->nbr_new += to.nbr_new;
        sum->bytes_alg += to.bytes_alg + so.bytes_alg;
    }
    return 0;
}

int gw_tick_result(gw_ctx* c, gw_tick_out* out) {
    if (!c || !out) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    return finish_tick(c, out);
}

int gw_synchronize(gw_ctx* c) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int gw_set_stream(gw_ctx* c, void* stream) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    HIPCHK(hipStreamSynchronize(c->st));
    c->st = stream ? (hipStream_t)stream : c->own_st;
    return 0;
}

}  // extern "C"
