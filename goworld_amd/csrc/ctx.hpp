// ctx.hpp — host-side state of one context (gw_ctx) shared by the C ABI
// translation units (capi.cpp: spaces, ticks, collects; world.cpp: RCCL
// communicator and the decomposed world).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "gw_internal.hpp"

namespace gw {
namespace host {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct SpaceHost {
    float d;
    uint32_t cap, base;
    SpaceP p;
    bool alive;
    uint32_t gen = 0;     // bumped by each destroy: a handle of the destroyed space no longer matches
};
// A space id handed to the caller: index | generation << SID_BITS.  A
// destroyed space's index is reused with the next generation, so a stale id
// (late destroy / grow / restore / set_ownership) is refused, never applied to
// the space that took its index (upstream spaces are keyed by unique EntityIDs,
// SpaceManager.go:21-27).
constexpr uint32_t SID_BITS = 20, SID_MASK = (1u << SID_BITS) - 1, SID_GEN_MASK = (1u << (32 - SID_BITS)) - 1;
inline uint32_t sid_handle(const SpaceHost& s, uint32_t idx) { return idx | ((s.gen & SID_GEN_MASK) << SID_BITS); }

struct OpSeg {            // submission order of a tick: host or device segment
    bool host;
    const gw_op* dev;
    const uint64_t* stamps;   // explicit global stamps (device) or nullptr
    uint32_t n;
    size_t host_off;
    const gw_halo_row* rows;  // halo rows (device): ops with inline stamps
};

struct Stage {
    const char* name;
    hipEvent_t a, b;
    uint64_t bytes;
};

// Decomposed world of this context (gw_world_*, world.cpp): one X-strip of one
// space, slots = global entity ids.
struct WorldHost {
    bool on = false;
    gw_world_geom g{};
    double h = 0;                   // halo width (dworld.Strips.h)
    uint32_t sid = 0;
    int nb[2] = {-1, -1};           // neighbour ranks (left, right), -1 = none
    float ext_lo[2] = {0, 0}, ext_hi[2] = {0, 0};   // their held x-ranges (float32)
    uint64_t tick = 0;              // world ticks routed (stamp layout)
    DevBuf stamps, send[2], recv[2], cnt;
    uint32_t send_cnt[2] = {0, 0}, recv_cnt[2] = {0, 0};   // entities (3 rows each)
    const gw_op* ops = nullptr;     // this tick's owned ops (caller's device memory)
    uint32_t n_ops = 0;
    bool routed = false;
    bool submitted = false;         // gw_world_submit queued a tick that gw_tick has not run yet
    uint32_t kept = 0;              // routed ops whose dedupe session (k_route1 = k_ops1) the tick ...
    uint32_t ol_pre = 0;            // ... reuses once submitted: the next tick's first ol_pre ops (gw_tick)
    uint32_t kept_tag = 0;          // that session
    // long moves (teleports): far triples, partitioned by destination rank
    DevBuf ext, far_rows, far_dest, far_cnt, far_sorted, far_off, far_cursor, far_recv, far_mat;
    uint32_t far_cap = 0;                        // triples the far buffer holds
    std::vector<uint32_t> far_cnt_h;             // [ranks + 1] triples this rank sends to each rank (incl.
                                                 // itself), then its long movers listed
    std::vector<uint32_t> far_off_h;             // [ranks] their offsets in far_sorted (triples)
    std::vector<uint32_t> far_mat_h;             // [ranks * (ranks + 1)] rank p's far_cnt vector (step path)
    // long-mover lists (group teleports): this rank's (longs, long_cap entries;
    // own_nlong after the last route), all ranks' (long_all) for the tick
    DevBuf longs, long_all;
    uint32_t long_cap = 0, own_nlong = 0;
    const gw_long_move* tick_longs = nullptr;    // queued for the next gw_tick (then cleared)
    uint32_t tick_nlong = 0;
    uint64_t conflicts_acc = 0;                  // long-mover conflicts of the ticks since gw_world_status
    std::vector<float> ext_h;                    // [2 * ranks] held x-range of every rank
    // host ops of a tick (gw_world_stage_ops): pinned staging, device copy, and
    // the event after the upload (the pinned buffer is reused once it fired)
    DevBuf hstage, dstage;
    hipEvent_t staged = nullptr;
    // the routing's counts after each route, written by one kernel into pinned
    // coherent host memory: [HaloStats | received counts (2) | far_cnt (R) | far_mat (R*R)]
    uint32_t* pub_h = nullptr;
    uint32_t* pub_d = nullptr;      // the same buffer as the device sees it
};

// transport (xport.cpp): one point-to-point transfer of an open group, and the
// loopback group of contexts driven by threads of one process
struct P2P {
    bool send;
    void* p;
    size_t bytes;
    int peer;
};
struct LocalGroup;

// a 16-byte EntityID as a hash-map key
struct Id16 {
    uint64_t a, b;
    bool operator==(const Id16& o) const { return a == o.a && b == o.b; }
};
struct Id16Hash {
    size_t operator()(const Id16& k) const {
        uint64_t h = k.a * 0x9E3779B97F4A7C15ull ^ (k.b + 0x632BE59BD9B4E019ull + (k.a << 6) + (k.a >> 2));
        return (size_t)(h ^ (h >> 29));
    }
};
inline Id16 id16(const void* p) {
    Id16 k;
    memcpy(&k, p, 16);
    return k;
}

}  // namespace host
}  // namespace gw

struct gw_ctx {
    using AoiEnt = gw::AoiEnt;
    using PrevEnt = gw::PrevEnt;
    using HaloStats = gw::HaloStats;
    using GEnt = gw::GEnt;
    using SpaceP = gw::SpaceP;
    using DevStats = gw::DevStats;
    using TickBufs = gw::TickBufs;
    using ScanCtx = gw::ScanCtx;
    using DevBuf = gw::host::DevBuf;
    using SpaceHost = gw::host::SpaceHost;
    using OpSeg = gw::host::OpSeg;
    using Stage = gw::host::Stage;
    int dev = 0;
    hipStream_t st = nullptr;
    hipStream_t own_st = nullptr;   // the context's own stream (st may be a caller's)
    // a collect that follows a deferred tick runs its flag / count / write
    // passes on st2 (after ev_diff: the tick's diff stage), beside the tick's
    // events stage on st; st waits for ev_col before the statistics publish
    hipStream_t st2 = nullptr;
    hipEvent_t ev_grid = nullptr, ev_diff = nullptr, ev_col = nullptr;
    ScanCtx sc2{};                  // the collect stream's look-back scans (sc is the tick's)
    int sw_halves = -1;             // GW_SW_HALVES: 1 / 0 force the write pass's half-wave mode, -1 automatic
    double rec_per_flagged = 1e9;   // records per flagged entity of the last collect (the mode's choice)
    bool overlap = true;            // GW_OVERLAP_COLLECT
    uint32_t overlap_min = 0;       // GW_OVERLAP_MIN: ... after ticks of at least this many ops (round 4: 65536,
                                    // a 1M world's 8-strip rank got 9 us slower with it; round 6, same box:
                                    // that rank 0.281 -> 0.272 ms, config #2 0.177 -> 0.162 ms with it)
    std::string err;

    std::vector<SpaceHost> spaces;
    uint32_t total_slots = 0, slot_cap = 0, total_cells = 0;
    // slot / cell ranges of destroyed (or moved) spaces, base -> length, all
    // below total_slots / total_cells and cleared: handed out first-fit
    std::map<uint32_t, uint32_t> free_slots, free_cells;
    uint32_t mpar = 0;                 // parity of the incremental grid rebuilds (TickBufs::mbit)
    uint16_t max_gate = 0;
    unsigned long long stamp_base = 1;   // global op counter (stamp 0 = never)
    uint32_t epoch = 1;                  // bumped by every tick and client change (World.nbc)
    static constexpr uint32_t PAIR_AUTO = 96, PAIR_MEAN = 128, PAIR_MOVERS = 131072;
    int cells_per_d = 2;                 // grid cells per AOI distance (GW_CELLS_PER_D)
    int diff_u = 1, nb_u = 4;            // k_mover waves per block (GW_MOVER_WPB), sync chunks in flight (GW_NB_U)
    bool grid_dirty = true;              // gn/gn_start must be rebuilt before queries
    uint64_t h_present = 0;
    uint64_t own_cap = 0;                // capacity of the own-event regions (grows on overflow)
    bool cells_zero = false;             // dep / arr / gm_cnt hold zeros

    // persistent device state (slot-indexed)
    gw::SlotRec* rec = nullptr;              // [slot_cap] AOI state, payload, pre-tick state, stamp, grid offset
    uint32_t* flags = nullptr;
    uint16_t* gate = nullptr;
    unsigned long long* nbc = nullptr;       // [slot_cap] epoch<<32 | neighbours with a client
    unsigned long long* nbg = nullptr;       // [slot_cap * 4] the same split by gate (World.nbg)
    uint32_t* movbit = nullptr;              // [slot_cap/32 + 1] movers of the tick, zero between ticks
    uint32_t* gmi = nullptr;                 // [slot_cap] primary mover-grid entry of a mover
    gw::OpLast* ol = nullptr;                // [slot_cap] per-op dedupe state (session-tagged words)
    uint32_t ol_tag = 0;                     // last dedupe session handed out (next_ol_tag)
    HaloStats* halo = nullptr;                // halo routing counters (device)
    GEnt* gnb[2] = {nullptr, nullptr};   // grid ping-pong (gnb[gcur] is current)
    uint32_t* gsb[2] = {nullptr, nullptr};  // cell starts ping-pong
    int gcur = 0;
    uint32_t cells_cap = 0;              // words in each per-cell array
    uint32_t *dep = nullptr, *arr = nullptr, *gm_cnt = nullptr, *cnt_new = nullptr, *dirty = nullptr,
             *gm_start = nullptr;
    SpaceP* sp_dev = nullptr;
    uint32_t sp_cap = 0;

    DevStats* stats = nullptr;     // device (grid rebuild, tick)
    bool stats_zero = true;        // stats is all zero (the last tick's reset pass, or init)
    DevStats* hstats = nullptr;    // pinned host (coherent): the tick's statistics, then the collect's (hcstats)
    DevStats* hstats_dev = nullptr;  // the same buffer as the device sees it
    DevStats* cstats = nullptr;    // device (collect: a deferred tick's stats stay intact)
    DevStats* hcstats = nullptr;   // pinned host

    // a tick launched but not read back yet (GW_TICK_DEFER): settled by the
    // next call that needs its results (the collect's one sync covers it)
    struct Pending {
        bool on = false, copied = false, reset_queued = false;
        uint32_t M = 0, C = 0, NC = 0, flags = 0;
        size_t s_grid = 0, s_movers = 0, s_diff = 0, s_events = 0;
        TickBufs b{};
    } pt;
    gw_tick_out last_out{};

    // grid + tick scratch
    DevBuf ops_buf, stamp_buf, k0, v0, k1, v1, gm, mtmp, mcell, cand, reg, pidx, heavy, rowrec, own, big, fall, mstat;
    DevBuf mir, ownc, mirc, mlist, mcnt, moff, minfo, icnt, ioff, mreg, chunk_first, srange, bk_a, bk_b, bk_id, bk_cnt, bk_split, ev_d, rtable;
    DevBuf scan_status, scan_status2, rs_hist, rs_os;   // rs_os: the one-kernel-per-pass sort's scratch (sort_u32_u32)
    uint32_t walk_min = 32;              // GW_WALK_MIN: TickBufs.walk_min (0: always walk)
    bool mover_compact = true;           // GW_MOVER_COMPACT: TickBufs.compact
    uint32_t heavy_min = 512;            // GW_HEAVY_MIN: TickBufs.heavy_min (0: off; 1M world at 8 strips:
                                         // diff 58 -> 47 us; round 6, config #3's 100k movers: diff 148 ->
                                         // 135 us, step -5..-8 us; rounds 3-4 measured cell order better there) ...
    uint32_t heavy_maxm = 262144;        // ... for ticks of at most GW_HEAVY_MAXM ops (round 4: 65536)
    uint32_t rank_sort = 12;             // GW_RANK_SORT: TickBufs.rank_sort
    // GW_DIRTY_SPAN: TickBufs.dirty_span; 0 = by the cell count: 2 up to 128k cells, 8 up to 1M cells (a hotspot wave
    // merges fewer dirty cells in a row: config #3 grid 63 -> 58 us), 16 above (fewer idle waves:
    // config #4's 4.4M cells at 4 per wave cost +50 us)
    uint32_t dirty_span = 0;
    uint32_t half_rows = 16;             // GW_HALF_ROWS: TickBufs.half_rows (tests of the fallback paths)
    uint32_t gate_lane_max = 255;        // GW_GATE_LANE_MAX: TickBufs.gate_lane_max (tests of the fallback)
    int32_t bk_flat = -1;                // GW_BK_FLAT, GW_POST_SPLIT, GW_PLACE_SPLIT: TickBufs' launch-merge knobs
    uint32_t post_split = 0, place_split = 0;
    bool dirty_split = false;            // GW_DIRTY_SPLIT=1: the dirty cells' merges in a launch of their own
    // GW_PAIR_MAX: TickBufs.pair_max (0: off, the default).  GW_PAIR_AUTO=1:
    // PAIR_AUTO when the last tick had >= PAIR_MOVERS movers averaging <=
    // PAIR_MEAN candidates (round 3: config #5 diff 1677 -> 1573 us with it;
    // round 6, same box, against k_mover_c: config #5 diff 1060 -> 1503 us,
    // step 3.62 -> 3.92 ms, a 16M-world strip's diff 136 -> 180 us)
    uint32_t pair_max = 0;
    bool pair_auto = false;
    uint64_t cand_mean = ~0ull;          // candidates per mover of the last tick
    uint32_t grid_cap = 0;               // GW_GRID_CAP: TickBufs.grid_cap (tests of the grid-stride loops)
    uint64_t ev_cap = 0;                 // events the flatten/sort buffers hold (grows on overflow)
    uint64_t ev_est = 0;                 // events expected this tick (last tick's count): sizes the buckets
    uint64_t it_est = 0;                 // bucket-path items of the last tick
    int ev_full_ticks = 0;               // ticks left on the general sort after a bucket overflowed
    int bk_overflows = 0;                // consecutive ticks whose buckets overflowed
    int bk_split_w = -1;                 // slot bits the bucket bounds were made for
    ScanCtx sc{};                  // single-pass scan state (prim.hpp)
    // sync / query scratch
    DevBuf fbits, flagged, rec_cnt, rec_off, rec0, rec1, gate_hist, gk0, gv0, gk1, gv1, qbuf;
    DevBuf cl_slot, cl_off, h_cl_slot, h_cl_off;   // GW_SYNC_BY_CLIENT segments (device / pinned host)
    DevBuf h_items;                               // gw_fanout's calls, staged in pinned memory
    DevBuf pay;                                   // per-client collect: payload per flagged entity
    uint64_t rec_cap = 0;                // records the rec0 buffer holds (grows on overflow)
    uint64_t flag_bound = 0;             // ops + restored slots since the last collect (>= flagged slots)
    // client messages (gw_client_events, gw_fanout): ping-pong + pinned host + gate offsets
    struct MsgBufs {
        DevBuf a, b, h;
        std::vector<uint64_t> goff;
    } m_create, m_destroy, m_fanout;
    DevBuf m_flag, m_at, m_items, m_cnt, m_off;
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
    int prof = 0;                      // 0 off, 1 every stage, 2 the "diff" stage only
    bool prof_cur = false;             // the stage being recorded is on
    std::vector<Stage> stages;
    size_t nstage = 0;
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;
    gw_stage_times last_times{};

    // ids, client-sync decode, wire encode (wire.cpp)
    std::unordered_map<gw::host::Id16, uint32_t, gw::host::Id16Hash> id_slot;   // entity id -> slot
    std::vector<gw::host::Id16> eid_h;       // [slot_cap] entity id of a slot (zero = none)
    std::vector<uint8_t> syncing_h;          // [slot_cap] SetClientSyncing
    uint4* eid_dev = nullptr;                // [slot_cap] 16-B entity ids
    uint4* cid_dev = nullptr;                // [slot_cap] 16-B client ids
    const gw_sync_record* last_rec = nullptr;   // records of the last collect (device)
    uint64_t last_R = 0;
    DevBuf wire_d, wire_h, wire_tab, id_up;
    std::vector<uint16_t> wire_gate;
    std::vector<uint64_t> wire_off;

    // communicator (xport.cpp: RCCL, or a loopback group of contexts of this
    // process) and decomposed world (world.cpp)
    ncclComm_t comm = nullptr;
    gw::host::LocalGroup* lgrp = nullptr;
    int c_nranks = 0, c_rank = 0;
    bool xp_open = false;                       // a transport group is being issued
    std::vector<gw::host::P2P> xp_pend;         // its transfers
    DevBuf xp_tmp;                              // loopback all-reduce scratch
    gw::host::WorldHost wd;
};

namespace gw {
namespace host {
int set_err(gw_ctx* c, int code, const char* fmt, ...);
int ensure(gw_ctx* c, DevBuf& b, size_t bytes);
int ensure_host(gw_ctx* c, DevBuf& b, size_t bytes);
int settle(gw_ctx* c);
int next_ol_tag(gw_ctx* c, uint32_t* tag);
int space_idx(gw_ctx* c, uint32_t handle, uint32_t* idx);   // a live space's index from its id (GW_ERANGE if stale)
World world_of(gw_ctx* c);
template <typename T>
T* P(DevBuf& b) { return (T*)b.p; }
// transport (xport.cpp): NCCL semantics on the context's stream, RCCL or loopback
bool xp_on(const gw_ctx* c);
int xp_group_start(gw_ctx* c);
int xp_send(gw_ctx* c, const void* p, size_t bytes, int peer);
int xp_recv(gw_ctx* c, void* p, size_t bytes, int peer);
int xp_group_end(gw_ctx* c);
void xp_abort(gw_ctx* c);                                   // drop an open group (error path)
int xp_allgather(gw_ctx* c, const void* send, void* recv, size_t bytes);   // `bytes` from every rank, rank order
int xp_allreduce_u64(gw_ctx* c, unsigned long long* dev, uint32_t n, int op);   // in place, GW_RED_*
void xp_release(gw_ctx* c);                                 // gw_shutdown
}  // namespace host
}  // namespace gw

#define HIPCHK(expr)                                                                             \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return gw::host::set_err(c, GW_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                     __FILE__, __LINE__);                                        \
    } while (0)
