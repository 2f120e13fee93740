// gw_internal.hpp — device data layout shared by the kernels and capi.cpp.
//
// Per context (one HIP device) the state of all spaces lives in one set of
// slot-indexed SoA arrays in HBM; a space owns a contiguous slot range and a
// contiguous range of uniform-grid cells, so one launch ticks every space of
// the device at once (BASELINE config #4: 10k spaces).
//
// There are no neighbour lists.  go-aoi's XZList relation of a pair is a pure
// function of the two current positions and of which member had the later AOI
// op: related(A,B) = inWin_c(other) where c has the larger
// global stamp.  Outside a one-ulp band around the window edge inWin_A(B) ==
// inWin_B(A) and the stamps do not matter, so they are only gathered there.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuaoi.h"

namespace gw {

// AOI state of one slot, 16 B (one dwordx4).  meta = space id | present<<31.
struct alignas(16) AoiEnt {
    float x, z;        // aoi.x, aoi.y of go-aoi == Position.X, Position.Z
    int32_t seq;       // unused (kept for the 16-B layout)
    uint32_t meta;
};
constexpr uint32_t PRESENT_BIT = 0x80000000u;
constexpr uint32_t SPACE_MASK = 0x7fffffffu;

// State of a mover before the tick, 16 B (written for this tick's movers).
// ox/oz are NaN when the slot was absent, so every window test against them
// fails.
struct alignas(16) PrevEnt {
    float ox, oz;
    unsigned long long ostamp;
};

// A slot's state in one 64-B record: an op, a collect or a resolve touches one
// line for all of it instead of one per array (AOI state, sync payload,
// pre-tick state, stamp, grid offset).
struct alignas(64) SlotRec {
    AoiEnt a;                  // AOI state
    float4 p;                  // x, y, z, yaw (sync payload)
    PrevEnt pv;                // pre-tick position and stamp (this tick's movers)
    unsigned long long stamp;  // global stamp of the slot's last AOI op
    uint32_t gidx;             // offset of the slot's entry inside its cell's range of gn
    uint32_t gate;             // World.gate[slot] again, read with the state (one line less per op / entity)
};
static_assert(sizeof(SlotRec) == 64, "SlotRec is one 64-B line");

// Per-slot op dedupe state, one 64-B record (a tick's op touches one line for
// all of it): the index of the slot's last op that sets the sync payload
// (non-Leave), its last AOI op, its last Leave, and per sync bit the last
// Leave that cleared it.  Each word is tag << 32 | op index, tag = the dedupe
// session (a tick, or a routing call whose tick reuses it); u64 atomicMax
// lets a newer session's index replace an older one and a word of an older
// session reads as -1 (ol_get), so nothing is reset between ticks.
struct alignas(64) OpLast {
    unsigned long long pos, aoi, leave, clr[2];
    unsigned long long rb[2];   // routing (halo.hip): the last non-Leave op setting sync bit c
    unsigned long long pad;
};
__device__ __forceinline__ unsigned long long ol_put(uint32_t tag, uint32_t i) {
    return ((unsigned long long)tag << 32) | i;
}
__device__ __forceinline__ int32_t ol_get(unsigned long long v, uint32_t tag) {
    return (uint32_t)(v >> 32) == tag ? (int32_t)(uint32_t)v : -1;
}

// Entry of the grid (cell-sorted, slot order inside a cell), 16 B.
struct alignas(16) GEnt {
    float x, z;
    uint32_t slot;     // DEPARTED: the entity left this cell during the tick being built
    uint32_t meta;     // cell | gate id (< 16) | CLIENT_BIT | MOVER_A / MOVER_B
};
// moved this tick (its pairs come from the mover grid): the tick's bit
// alternates between ticks (TickBufs::mbit), and the grid rebuild of the next
// tick drops the other one while it copies the entries (no clearing pass)
constexpr uint32_t MOVER_A = 0x80000000u;
constexpr uint32_t MOVER_B = 0x20000000u;
constexpr uint32_t CLIENT_BIT = 0x40000000u;   // has a client (GameClient != nil)
constexpr uint32_t CELL_MASK = 0x01ffffffu;    // cells of a context: < 2^25 (capi.cpp)
// the client's gate id when it is below 16 (a collect with at most 16 gate
// ids reads a watcher's gate from its grid entry, no gather of gate[slot])
constexpr uint32_t NBC_GATES = 0x80000000u;    // nbc low word: nbg holds the per-gate split (World.nbg)
constexpr uint32_t NBC_COUNT = 0x7fffffffu;
constexpr int GATE_SHIFT = 25;
constexpr uint32_t GATE_MASK = 0xfu << GATE_SHIFT;
__host__ __device__ inline uint32_t gate_meta(uint32_t gate) {
    return gate ? (CLIENT_BIT | ((gate < 16u ? gate : 0u) << GATE_SHIFT)) : 0u;
}
constexpr uint32_t DEPARTED = 0xffffffffu;
constexpr uint32_t CELL_DIRTY = 0x80000000u;   // flag in dep[c]: the cell is re-sorted this tick

// Entry of the mover grid, 32 B: a mover appears at the cell of its old
// position (TAG_OLD) and at the cell of its new one (TAG_NEW), once with both
// tags when the two cells agree.  Both positions travel with every entry.  The
// TAG_PRIMARY entry (the new one, or the old one of a leaver) is where the
// mover's own diff runs, so movers are processed in cell order.
struct alignas(16) MEnt {
    float x, z, ox, oz;          // NaN when absent after / before the tick
    uint32_t slot, tags, client, space;
};
constexpr uint32_t TAG_OLD = 1u, TAG_NEW = 2u, TAG_PRIMARY = 4u;
constexpr uint32_t TAG_LONG = 8u;   // decomposed world: the mover jumped further than max_step this tick

// Per-space parameters (32 B).  Cells are squares of side cs = 1/inv_cs >=
// d / cells_per_d; a window spans at most 10 rows (capi.cpp).  The cell
// function is monotone in x and z, which keeps the candidate search exact
// whatever the float rounding.
struct alignas(16) SpaceP {
    float d;
    float x0, z0, inv_cs;
    int32_t W, H;
    uint32_t cell_base;
    uint32_t alive;
    float own_lo, own_hi;      // ownership x-range (decomposed world), default (-inf, +inf)
    float pad0, pad1;
};
__device__ __forceinline__ bool owned_x(const SpaceP& P, float x) { return x >= P.own_lo && x < P.own_hi; }

constexpr int STAT_SHARDS = 256;
constexpr int SH_FIELDS = 4;
constexpr int SH_MOVERS = 0;  // distinct slots with an AOI op (k_ops3)
constexpr int SH_AOLD = 1;    // a_old | a_new << 32 (per-shard sums stay below 2^32)

// Device-side counters of one tick / collect (read back once per call).
// a collect with at most this many gate ids (0 = no client included) writes
// each record straight into its gate's partition (count and write passes per
// (gate, entity); no sort, no second host sync)
constexpr uint32_t GATE_DIRECT_MAX = 16;
struct DevStats {
    unsigned long long n_present;     // entities in the grid
    unsigned long long n_movers;      // unused (movers are counted in shard[][SH_MOVERS])
    unsigned long long cand_total;    // sum of candidate bounds over movers
    unsigned long long n_gm;          // mover-grid entries
    unsigned long long ev_pk;         // sum of (enters | leaves<<32) over watchers
    unsigned long long n_big;         // own-event segments left for the block sort
    unsigned long long n_mlist;       // movers with events (slot-ordered list)
    unsigned long long n_sort;        // events (general sort) / items (bucket path) flattened
    unsigned long long n_items;       // bucket path: items of the listed movers
    unsigned long long bk_tiles;      // bucket path: tiles in use (count table stride)
    unsigned long long bk_cells;      // bucket path: count table entries in use
    unsigned long long overflow;      // event regions exceeded their capacity
    unsigned long long bk_max;        // largest event bucket too big for the LDS sort (0: none)
    unsigned long long bad_ops;
    unsigned long long flagged;       // sync: flagged entities
    unsigned long long rec_total;     // sync: records
    unsigned long long n_heavy;       // heavy-first k_mover: primaries with >= heavy_min candidates (heavy[])
    unsigned long long n_fall;        // small-space diff: mover-grid entries left to k_mover_list (fall[])
    unsigned long long n_conflicts;   // decomposed world: long-mover pairs the lists did not cover (this
                                      // attempt; folded into the world's counter once per tick by the host)
    unsigned long long gate_base[GATE_DIRECT_MAX];   // sync, several gates: first record of gate g (gate_off)
    unsigned long long shard[STAT_SHARDS][SH_FIELDS];   // per-field sums in shard[0] on the host
};

// ---- primitives (prim.hpp; host wrappers in sync.hip) -----------------------
// State of the single-pass scans of one context (one stream): the tile status
// words, the monotonic tile ticket, and the host-side ticket base and tag.
struct ScanCtx {
    unsigned long long* status;   // [max_tiles * scan_words()]
    unsigned long long* ticket;   // one word, never reset
    unsigned long long tbase;     // tickets handed out by earlier scans
    uint32_t tag;                 // tag of the last scan (status words of other tags are stale)
    uint64_t max_tiles;
};
struct RadixTmp {
    uint32_t* hist;      // 256 * radix_blocks(n_max)
    ScanCtx* sc;
    uint32_t* os = nullptr;   // radix2_scratch(n_max) words: sort_u32_u32 runs radix_sort2 (one kernel per pass)
};
uint64_t radix_tile();            // keys per radix block
uint64_t radix2_tile();           // keys per tile of radix_sort2
uint64_t radix2_scratch(uint64_t n_max);   // u32 scratch words of radix_sort2
uint64_t scan_tile();             // elements per scan tile
uint64_t scan_words();            // status words per scan tile
void scan_u32_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint32_t* total, hipStream_t s);
void scan_u32_u64(const uint32_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint64_t* total, hipStream_t s);
void scan_u64_u64(const uint64_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                  uint64_t* total, hipStream_t s);
// stable sort of packed pairs (u64: value << 32 | key) by key bits [lo_bit, hi_bit); 1 = result in p1
int sort_pairs64(uint64_t* p0, uint64_t* p1, uint64_t n_max, const uint64_t* n_dev, int lo_bit, int hi_bit,
                 RadixTmp& tmp, hipStream_t s);
int sort_u32_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                 int lo_bit, int hi_bit, RadixTmp& tmp, hipStream_t s);

// ---- persistent per-context state -----------------------------------------
struct World {
    uint32_t cap;              // total slots
    uint32_t ncells;
    const SpaceP* sp;
    SlotRec* rec;              // [cap] per-slot state
    uint32_t* flags;           // syncInfoFlag, packed: 2 bits per slot, 16 slots per word (flag_word / flag_sh)
    uint16_t* gate;            // client gate, 0 = no client
    GEnt* gn;                  // [cap] current grid, n_present entries
    uint32_t* gn_start;        // [ncells+1] first entry of each cell
    // |{w related to e : w has a client}| as of the end of tick `epoch`
    // (epoch<<32 | count), written for every present mover by the diff; a
    // collect right after that tick takes it instead of walking e's window
    unsigned long long* nbc;
    // with NBC_GATES set in nbc[e]: nbg[4e .. 4e+3] = the same count split by
    // the watchers' gate ids (16 bits per gate, gate g in word g / 4 at bit
    // 16 * (g % 4)), written by k_mover_c in a context with 2 < G <= 16
    unsigned long long* nbg;
    uint32_t epoch;            // current epoch (bumped by every tick and client change)
    int nb_u;                  // candidate chunks of 64 in flight in the sync walks
};

// rows of a mover's rectangles whose index ranges k_bounds hands to k_mover
constexpr uint32_t RR_ROWS = 8;

// ---- tick buffers handed to the launchers ----------------------------------
// k_bounds tags each primary mover-grid entry's candidate bound with PRIM_ONE,
// so the scan of the bounds also counts the primaries before each entry (its
// index among them) and their total; readers of cand / reg mask with CAND_MASK
constexpr int PRIM_SHIFT = 36;
constexpr uint64_t PRIM_ONE = 1ull << PRIM_SHIFT;
constexpr uint64_t CAND_MASK = PRIM_ONE - 1;

struct TickBufs {
    World w;                  // gn / gn_start: the grid before the tick (the new one from tick_movers on)
    const gw_op* ops;
    const unsigned long long* stamps;   // explicit global stamps (nullptr: stamp_base + index)
    uint32_t m;               // ops in the stream
    uint32_t op0;             // ops [0, op0) were deduped into ol by the world's routing (k_ops1 starts here)
    unsigned long long stamp_base;
    OpLast* ol;               // [cap] per-slot op dedupe state (words of this tick's session ol_tag)
    uint32_t ol_tag;          // the tick's dedupe session
    uint32_t mbit, mstale;    // this tick's mover bit (MOVER_A / MOVER_B) and the last tick's
    DevStats* st;
    // incremental grid: gn -> gn_nxt
    GEnt* gn_nxt;             // [cap]
    uint32_t* start_nxt;      // [ncells+1]
    uint32_t* dep;            // [ncells] departures (| CELL_DIRTY), zero between ticks
    uint32_t* arr;            // [ncells] arrivals, zero between ticks
    uint32_t* cnt_new;        // [ncells+1] entries per cell after the tick
    // mover grid (counting sort by cell; gm_cnt is zero between ticks)
    uint32_t* gm_cnt;         // [ncells+1]
    uint32_t* gm_start;       // [ncells+1]
    MEnt* gm;                 // [2m]
    MEnt* mtmp;               // [m] op i's mover-grid entry (tags aside) when op i is a mover (k_ops3 -> k_place)
    uint4* mcell;             // [m] op i: old / new cell of its mover (NO_CELL: none), slot, syncInfoFlag bits to OR
    // diff (indexed by mover-grid entry)
    uint64_t* cand;           // [2m] candidate bound (0 unless TAG_PRIMARY) | PRIM_ONE if primary
    uint64_t* reg;            // [2m] exclusive scan of cand: region offset | primaries before << PRIM_SHIFT
    uint32_t* pidx;           // [m] k-th primary entry (written by the scan of cand; k_mover's waves)
    uint32_t* heavy;          // [m] heavy-first mode: primaries with >= heavy_min candidates, walked first
    uint32_t heavy_min;       // GW_HEAVY_MIN (0: off): longest walks first when few movers (shorter tail)
    uint4* rowrec;            // [2m * RR_ROWS] per primary entry: its rows' grid / mover-grid index ranges
                              // (start, end, start, end) from k_bounds; row 0 = (1, 0, ..) when > RR_ROWS rows
    uint64_t own_cap;         // capacity of own / mir
    uint32_t* own;            // own events (target<<1 | leave), sorted by target per mover
    uint64_t* mir;            // mirror events of op-less neighbours: watcher<<32 | mover<<1 | leave
    unsigned long long* ownc; // [2m] own enters | leaves<<32 per entry
    unsigned long long* mirc; // [2m] mirror enters | leaves<<32 per entry
    unsigned long long* mstat;   // [2m] A_old | A_new << 32 per entry (k_mover -> k_mover_post)
    uint32_t* big;            // [2m] entries whose own events need the block sort
    uint32_t* fall;           // [2m] small-space mode: entries the half-wave walk could not take (k_mover_list)
    // canonical events: movers in slot order, their events flattened, one
    // stable radix sort by (leave, watcher) -> (watcher, target) order
    uint32_t* movbit;         // [cap/32 + 1] movers, zero between ticks
    uint32_t* gmi;            // [cap] primary mover-grid entry of a mover slot
    uint32_t* mlist;          // [m] movers in slot order
    unsigned long long* mcnt; // [m] all events of a listed mover (enters | leaves<<32)
    unsigned long long* moff; // [m] exclusive scan of mcnt
    uint4* minfo;             // [m] listed mover: slot, own enters, own leaves, mirror events
    uint32_t* icnt;           // [m] bucket path: items of a listed mover (own runs + mirror events)
    uint32_t* ioff;           // [m] exclusive scan of icnt
    unsigned long long* mreg; // [m] its region offset
    uint32_t* chunk_first;    // [ev_cap / 64] listed mover holding flat position 64c
    uint32_t *fk0, *fv0, *fk1, *fv1;   // [ev_cap] general sort: key leave<<wbits | watcher, value target
                                       // (aliases of bk_a / bk_b)
    uint64_t *bk_a, *bk_b;    // [ev_cap] bucket path: (leave<<wbits | watcher) << 32 | target
    uint16_t* bk_id;          // [ev_cap] bucket of each flat event
    unsigned long long* bk_cnt;   // [NB * bk_tiles] per (bucket, tile) items | events<<32, scanned in place
    uint32_t bk_tiles;        // tiles of BK_TILE flat positions covering ev_cap
    uint32_t* bk_split;       // [BK_NSPLIT] bucket bounds: quantiles of the last tick's keys
    int bk_bits;              // log2 of the bucket count (<= BK_MAXBITS, <= wbits + 1)
    uint64_t it_hint;         // bucket-path items of the last tick (sizes the flatten's grid)
    float long_step;          // decomposed world: an owned mover whose x moves further is a long
                              // mover (its pairs are attributed to the targets' owners); +inf otherwise
    const gw_long_move* longs;   // decomposed world: every rank's long movers of the tick (group teleports:
    uint32_t n_long;             // their pairs are evaluated from these by the owner of the watcher)
    uint32_t gate_counts;     // G when 2 < G <= GATE_DIRECT_MAX (k_mover_c splits nbc by gate, World.nbg), else 0
    unsigned long long* conflicts;   // decomposed world (else null; DevStats.n_conflicts): long-mover pairs the lists did not
                                     // cover (no list queued, or the watcher missing from it), HaloStats
    uint32_t dirty_span;      // GW_DIRTY_SPAN: cells whose dirty flags one k_grid_dirty wave scans (1..64)
    // launch-merge knobs (A/B and tests; gw_ctx reads them at gw_init): GW_BK_FLAT (-1 automatic,
    // 0 / 1: the bucket items made by k_flat_items / the count pass), GW_POST_SPLIT (k_mover_post
    // in a launch of its own), GW_PLACE_SPLIT (k_place and k_grid_copy apart)
    int32_t bk_flat;
    uint32_t post_split, place_split;
    uint32_t compact;         // GW_MOVER_COMPACT (default 1): k_mover runs one wave per primary entry
                              // (pidx), else one per mover-grid entry, the others exiting
    uint32_t pair_max;        // GW_PAIR_MAX: k_mover_pair runs two movers per wave when both have at
                              // most this many candidates (0 = one mover per wave, k_mover)
    uint32_t grid_cap;        // GW_GRID_CAP (tests): at most this many blocks for the grid-stride
                              // flatten / bucket tile passes (0 = no cap)
    int ev_full;              // 1: general stable radix sort instead of the bucket path
    gw_event* ev;             // [ev_cap] canonical events, enters then leaves
    uint64_t ev_cap;
    uint32_t* rtable;         // radix_sort2 scratch
    int wbits;                // bits of a slot
    uint32_t n_spaces;        // spaces of the context (dead ones included)
    uint32_t small_ents;      // small-space mode: max entries per space (0: off)
    uint32_t small_cells;     //   and max cells per space
    int small_halves;         //   two movers per wave (GW_MOVER_HALVES, default on)
    uint32_t half_rows;       //   rows a half-wave walk takes (16; GW_HALF_ROWS lowers it in tests: more
                              //   pairs left to mover_one / k_mover_list)
    uint32_t gate_lane_max;   // per-gate split: a lane's client count up to which it is exact (255, the
                              // 8-bit counters; GW_GATE_LANE_MAX lowers it in tests: more walked entries)
    int diff_u;               // candidate chunks of 64 in flight per k_mover iteration
    uint32_t walk_min;        // mean candidates per row range from which a walk maps chunks by readlanes
    uint32_t rank_sort;       // own events sorted by rank (readlanes) up to this many, more by a network
};

// events bucket path (aoi.hip k_flat_count / k_bucket_scatter / k_bucket_sort)
constexpr int BK_NT = 1024;           // threads of the tile kernels
constexpr int BK_TILE = 8192;         // flat positions per tile
constexpr int BK_MAXBITS = 12;        // at most 4096 buckets
constexpr int BK_LCAP = 3584;         // items a bucket may hold (LDS sort; 3.5x the mean: 44 KB of LDS, 3 blocks per CU)
constexpr int BK_SNT = 512;           // threads of the bucket sort
constexpr int BK_HBINS = 2048;        // bins of the counting sort inside a bucket
constexpr int BK_SHORT = 16;          // longer bins are sorted by a wave
constexpr int BK_RUNS = 512;          // own runs a bucket copies block-wide (more: by their lane); == BK_SNT
constexpr uint64_t BK_MEAN = 1024;    // target mean bucket size when choosing bk_bits (2048 with 7168: +6 us at config #3)
constexpr uint32_t BK_NSPLIT = 1u << BK_MAXBITS;   // quantile table size
// item bits: (leave, watcher, target) = 2*wbits + 1 <= BK_KEY_BITS, then the
// run flag, then (staged only) the bucket in the top BK_MAXBITS bits
constexpr int BK_KEY_BITS = 51;
constexpr int BK_MAX_WBITS = (BK_KEY_BITS - 1) / 2;   // 25: larger contexts take the general sort
static_assert(BK_KEY_BITS + 1 + BK_MAXBITS <= 64, "item layout");
void launch_bk_split_init(uint32_t* sp, int wbits, hipStream_t s);

// ---- launchers --------------------------------------------------------------
// full rebuild of the grid (spaces created, first use): stable radix sort of
// (cell, slot) pairs into w.gn / w.gn_start; k0..v1 hold cap keys each
void grid_rebuild(const World& w, DevStats* st, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1,
                  RadixTmp& rt, int key_bits, hipStream_t s);
// one tick, in launch order (device-side counts only: no host sync inside)
void tick_ops(const TickBufs& b, hipStream_t s);
// gn -> gn_nxt, start_nxt (dirty = false: the dirty cells' merges are left to tick_movers)
void tick_grid(const TickBufs& b, ScanCtx& sc, hipStream_t s, bool dirty = true);
// b.w: the new grid; pre: the buffers before the flip, whose dirty cells it
// merges in the bounds' launch (tick_grid ran with dirty = false)
void tick_movers(const TickBufs& b, ScanCtx& sc, hipStream_t s, const TickBufs* pre = nullptr);
void tick_diff(const TickBufs& b, hipStream_t s);                  // own + mirror events per mover
void tick_events(const TickBufs& b, ScanCtx& sc, hipStream_t s);   // canonical event arrays
// after the host read the counts (given by value); zeroes the tick's DevStats
// the per-tick reset (next tick's bucket bounds, zeroed statistics): one block
constexpr int RESET_NT = 1024;
void tick_reset(const TickBufs& b, hipStream_t s);
// bytes (multiple of 8) from device src to a device-visible pinned host buffer
// by one kernel, then the reset of tick *b unless b is null
void publish_stats(const TickBufs* b, const void* src, void* host_dst, size_t bytes, hipStream_t s);
// up to 4 device ranges of u32 words into device-visible pinned host memory by
// one kernel (instead of a blit copy each): the world's routing counts
struct PubSeg {
    const uint32_t* src;
    uint32_t* dst;
    uint32_t words;
};
void publish_words(const PubSeg* segs, int n, hipStream_t s);

void launch_set_clients(const World& w, const uint32_t* slots, const uint16_t* gates, uint32_t n, bool grid_ok,
                        hipStream_t s);
// sync collect
void launch_sync_write_small(const World& w, uint32_t n_spaces, const uint32_t* flagged, const uint32_t* fbits,
                             const uint64_t* rec_off, const uint32_t* cnt, gw_sync_record* rec, uint64_t rec_cap,
                             DevStats* st, const uint32_t* sfirst, const uint32_t* slast, uint32_t max_ents,
                             uint32_t max_cells, hipStream_t s);
// small-space mode: every space's grid (entries + row starts) in this many LDS bytes at most
constexpr size_t SMALL_LDS_MAX = 48 * 1024;
// also zeroes *ovf, the write passes' overflow flag (the collect's only
// accumulated counter: no reset copy of the collect's DevStats), and zero[0, nzero)
void launch_flag_compact(uint32_t* flags, uint32_t cap, uint32_t* flagged, uint32_t* fbits, ScanCtx& sc,
                         unsigned long long* total, unsigned long long* ovf, uint32_t* zero, uint32_t nzero,
                         hipStream_t s);
// sfirst / slast (small-space mode, else null): each space's run of the flagged list
void launch_sync_count(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, uint32_t* cnt, uint32_t* sfirst, uint32_t* slast, hipStream_t s);
// several gates (G <= GATE_DIRECT_MAX): counts per (gate, entry), gate-major
// cnt[g * nf_max + k]; then, after their exclusive scan off, every record at
// its gate's position (sync.hip)
void launch_sync_gates(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, uint32_t G, uint32_t* cnt, hipStream_t s);
void launch_sync_write_gates(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                             uint32_t nf_max, uint32_t G, const uint64_t* off, gw_sync_record* rec, uint64_t rec_cap,
                             DevStats* st, hipStream_t s);
void launch_sync_write(const World& w, const uint32_t* flagged, const uint32_t* fbits, const uint64_t* nf_dev,
                       uint32_t nf_max, const uint64_t* rec_off, const uint32_t* cnt, gw_sync_record* rec,
                       uint64_t rec_cap, DevStats* st, hipStream_t s,
                       uint64_t* pairs = nullptr, float4* pay = nullptr, bool halves = false);
// the records and the client segment table in one pass (k_records_seg)
void launch_records_seg(const World& w, const uint64_t* pairs, const uint32_t* idx, const uint32_t* flagged, const float4* pay, uint64_t n, gw_sync_record* out,
                        uint32_t* client_slot, uint64_t* client_off, uint32_t* n_clients, ScanCtx& sc,
                        hipStream_t s);
void launch_gate_hist(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* hist /*65536*/, hipStream_t s);
void launch_gate_keys(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* keys, uint32_t* vals, hipStream_t s);
void launch_gather_records(const gw_sync_record* in, const uint32_t* idx, const uint64_t* n_dev,
                           uint64_t n_max, gw_sync_record* out, hipStream_t s);
// queries
void launch_neighbors(const World& w, uint32_t slot, uint32_t* out, uint32_t* n_out, uint32_t cap, hipStream_t s);
void launch_count_all(const World& w, uint64_t n_present, unsigned long long* total, hipStream_t s);
// ---- decomposed world: owner-side halo routing (halo.hip) -----------------
constexpr uint8_t SIF_ROUTED = GW_SIF_OWN_CLIENT | GW_SIF_NEIGHBOR_CLIENTS;   // flag bits rows carry
// the first three words are summed over ranks by gw_world_status
struct HaloStats {
    unsigned long long overflow;    // routed entities past a fixed-size buffer (0 by construction)
    unsigned long long conflicts;   // pairs of long movers related before or after a tick (the diff)
    unsigned long long bad_ops;     // ops with an invalid slot or kind
    unsigned long long long_moves;  // owned entities that moved more than max_step (routed far)
    uint32_t cnt[2];                // entities placed per neighbour destination (this call)
    uint32_t far_n;                 // far triples placed (this call; may exceed the buffer)
    uint32_t long_n;                // long movers listed (this call; may exceed the list buffer)
};
// halo rows of long moves (teleports): to every rank holding the old or the
// new position that is not a neighbour, and a LEAVE for the owner's own copy
// when the entity left its held range.  Triples in placement order with
// their destination rank (partitioned by destination afterwards).
struct HaloFar {
    gw_halo_row* rows;          // cap triples (3 rows each)
    uint32_t* dest;             // destination rank of each triple
    uint32_t* cnt;              // [nranks + FAR_EXTRA] triples per destination, the long movers listed,
                                // a pad word, the entities routed to the left / right neighbour
                                // (zeroed by the first pass; all-gathered as one vector at >= 3 ranks)
    const float* ext;           // [2 * nranks] held x-range [lo, hi) of every rank, float32
    uint32_t cap, nranks, self, pad;
    gw_long_move* longs;        // [long_cap] this rank's long movers (group teleports), or null
    uint32_t long_cap, pad2;
};
constexpr uint32_t FAR_EXTRA = 4;  // HaloFar::cnt words after the per-rank triples
constexpr uint16_t RES_LONG = 1;   // gw_op.reserved of a halo row: the entity moved more than max_step
struct HaloDst {
    float x_lo, x_hi;
    gw_halo_row* rows;
    uint32_t cap;
};
struct HaloDsts {
    HaloDst d[2];
    uint32_t n;
};
// ol_tag: the routing's dedupe session (a tick that reuses it passes the same tag).
// stamps_out != nullptr: the first pass also writes stamps_out[i] = stamp_base + i
// (then `stamps` may be stamps_out); pad: NOP rows up to each buffer's capacity
void launch_route_halo(const World& w, const gw_op* ops, const unsigned long long* stamps, uint32_t n,
                       float max_step, const HaloDsts& D, OpLast* ol, uint32_t ol_tag, HaloStats* hs, hipStream_t s,
                       bool pad = true, unsigned long long* stamps_out = nullptr, unsigned long long stamp_base = 0,
                       const HaloFar* far = nullptr);
// far triples -> out, grouped by destination: triple t goes to off[dest[t]] + (its rank among them);
// cursor: [nranks] scratch, overwritten
void launch_far_partition(const gw_halo_row* rows, const uint32_t* dest, uint32_t n, const uint32_t* off,
                          uint32_t* cursor, uint32_t nranks, gw_halo_row* out, hipStream_t s);
void launch_iota_u64(unsigned long long* p, unsigned long long base, uint32_t n, hipStream_t s);
// out[i] = sum (mx: max) over r < R of in[r * n + i]
void launch_reduce_u64(const unsigned long long* in, unsigned long long* out, uint32_t n, uint32_t R, bool mx,
                       hipStream_t s);
// up to SEG_MAX device segments of a tick's op stream (halo rows, or ops with
// stamps when the tick is stamped) gathered by one launch
constexpr int SEG_MAX = 8;
struct SegTable {
    struct Seg {
        const gw_op* ops;
        const unsigned long long* stamps;
        const gw_halo_row* rows;
        uint32_t off;
    } seg[SEG_MAX];
    uint32_t n, total;
};
void launch_gather_segs(const SegTable& t, gw_op* ops, unsigned long long* stamps, hipStream_t s);
void launch_split_rows(const gw_halo_row* rows, uint32_t n, gw_op* ops, unsigned long long* stamps,
                       hipStream_t s);
void launch_watcher_keys(const gw_sync_record* rec, uint64_t n, uint32_t* keys, uint32_t* vals, hipStream_t s);
void launch_client_segments(const gw_sync_record* rec, uint64_t n, uint32_t* head, uint32_t* pos,
                            uint32_t* n_clients, uint32_t* client_slot, uint64_t* client_off, ScanCtx& sc,
                            hipStream_t s);
void launch_restore(const World& w, const uint32_t* slots, const float4* xyzw, uint32_t n,
                    unsigned long long stamp_base, uint32_t flags, hipStream_t s);
// client messages (sync.hip)
// client messages of n events in one look-back pass; the count to *n_out
void launch_event_client_compact(const gw_event* ev, uint64_t n, const uint16_t* gate, const SlotRec* rec,
                                 uint32_t* out, bool create, uint32_t* n_out, ScanCtx& sc, hipStream_t s);
// out == nullptr: counts per item into cnt; else deliveries at off[k]
void launch_fanout(const World& w, const uint32_t* items, uint32_t n, uint32_t* cnt, const uint64_t* off,
                   uint64_t* pairs, hipStream_t s);
void launch_fanout_final(const uint64_t* pairs, const uint32_t* idx, const uint32_t* items, uint64_t n,
                         gw_fanout_rec* out, hipStream_t s);
// keys[i] = gate[w[i]], vals[i] = i, hist[gate] += 1 (hist zeroed by the caller)
void launch_gate_keys(const uint64_t* pairs, const uint16_t* gate, uint64_t n, uint32_t* keys, uint32_t* vals,
                      uint32_t* hist, hipStream_t s);
void launch_msg_keys(const uint32_t* rec, int words, uint64_t n, const uint16_t* gate, uint32_t* keys, uint32_t* vals,
                     hipStream_t s);   // gate == nullptr: key = watcher
void launch_msg_gate_hist(const uint32_t* rec, int words, uint64_t n, const uint16_t* gate, uint32_t* hist,
                          hipStream_t s);
void launch_msg_gather(const uint32_t* in, int words, const uint32_t* idx, uint64_t n, uint32_t* out,
                       hipStream_t s);
void launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);
// ids and the wire encode (sync.hip)
void launch_put16(uint4* table, const uint32_t* slots, const uint4* vals, uint32_t n, hipStream_t s);
struct WirePacket {              // one gate's packet of the wire encode
    uint64_t rec0, nrec;         // its records in the collect's stream
    uint64_t byte_off;           // packet offset in the output
    uint32_t gate, pad;
};
void launch_wire_encode(const gw_sync_record* rec, uint64_t R, const WirePacket* pk, uint32_t npk,
                        const uint4* eid, const uint4* cid, uint32_t* out, hipStream_t s);
void launch_fill_i32(int32_t* p, int32_t v, uint64_t n, hipStream_t s);
// space lifecycle (space.hip): move a slot range's state, clear a range, count present entities
void launch_slots_move(const World& w, OpLast* ol, uint4* eid, uint4* cid, uint32_t src, uint32_t dst, uint32_t n,
                       hipStream_t s);
void launch_slots_clear(const World& w, OpLast* ol, uint4* eid, uint4* cid, uint32_t base, uint32_t n,
                        uint32_t meta, hipStream_t s);
void launch_count_present(const SlotRec* rec, uint32_t base, uint32_t n, unsigned long long* out, hipStream_t s);

}  // namespace gw
