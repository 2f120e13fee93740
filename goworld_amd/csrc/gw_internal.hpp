// gw_internal.hpp — device data layout shared by kernels.hip and capi.cpp.
//
// Per context (one HIP device) the state of all spaces lives in one set of
// slot-indexed SoA arrays in HBM; a space owns a contiguous slot range and a
// contiguous range of uniform-grid cells, so one launch ticks every space of
// the device at once (BASELINE config #4: 10k spaces).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuaoi.h"

namespace gw {

// AOI state of one slot, 16 B (one dwordx4).  meta = space id | present<<31.
struct alignas(16) AoiEnt {
    float x, z;        // aoi.x, aoi.y of go-aoi == Position.X, Position.Z
    int32_t seq;       // index of the slot's last AOI op in the current tick, -1 otherwise
    uint32_t meta;
};
constexpr uint32_t PRESENT_BIT = 0x80000000u;
constexpr uint32_t SPACE_MASK = 0x7fffffffu;

// Entity in the cell-sorted grid array, 16 B.
struct alignas(16) SortEnt {
    float x, z;
    uint32_t slot;
    int32_t seq;
};

// Neighbour list of one slot (InterestedIn == InterestedBy), 16 B.  The list
// lives in a pool region of 2*cap entries split in two halves: the current
// list is at `cur`, the next tick's list is written to `alt` and the halves
// swap, so no list is ever rewritten in place.  Lists are ascending slots.
struct alignas(16) LstMeta {
    uint32_t cur, alt, cnt, cap;
};

// Per-space parameters (32 B).  Cells are squares of side cs = 1/inv_cs >= d:
// a window spans at most 3x3 cells.  The cell function is monotone in x and z,
// which keeps the candidate search exact whatever the float rounding.
struct alignas(16) SpaceP {
    float d;
    float x0, z0, inv_cs;
    int32_t W, H;
    uint32_t cell_base;
    uint32_t alive;
};

constexpr int STAT_SHARDS = 256;
constexpr int SH_FIELDS = 8;
constexpr int SH_PAIRS = 0, SH_AOLD = 1, SH_ANEW = 2, SH_REALLOC = 3, SH_MAT = 4, SH_LOGAPP = 5, SH_MERGE = 6;

// Delta log of one slot: up to LOGCAP pending events (target<<1 | leave) of an
// op-less watcher, applied to its sorted list lazily (when it moves, is
// collected, is queried or the log fills).  Lists are the base list plus the
// log's net effect.
constexpr uint32_t LOGCAP = 128;

// Device-side counters of one tick / collect (read back once per call).
struct DevStats {
    unsigned long long n_present;     // entities in the grid
    unsigned long long movers_present;
    unsigned long long leavers;
    unsigned long long bound_pk;      // sum of (cand | old<<32) over movers
    unsigned long long tier_pk;       // count of (tierS | tierB<<32)
    unsigned long long n_tier_c;
    unsigned long long tier_c_temp;   // u32 words of tier-C scratch
    unsigned long long ev_pk;         // sum of (enters | leaves<<32) over watchers
    unsigned long long n_affected;    // non-mover watchers with events
    unsigned long long n_bigseg;      // watchers whose event segments need the block sort
    unsigned long long bigseg_temp;   // u32 words of big-segment scratch
    unsigned long long pool_top;      // bump pointer of the neighbour pool (entries)
    unsigned long long pool_overflow;
    unsigned long long tmp_overflow;
    unsigned long long bad_ops;
    unsigned long long pairs_tested, a_old, a_new, reallocs;   // reduced from shards
    unsigned long long materialized, log_appends, seg_merges;
    unsigned long long flagged;       // sync: flagged entities
    unsigned long long rec_total;     // sync: records
    unsigned long long scratch;       // generic scan total sink
    unsigned long long shard[STAT_SHARDS][SH_FIELDS];
};

// ---- primitives (instantiated in kernels.hip) ------------------------------
struct RadixTmp {
    uint32_t* hist;      // 256 * radix_blocks(n_max)
    uint32_t* scan_tmp;  // scan_tmp_elems(256 * radix_blocks(n_max))
    uint32_t* scan_total;
};
uint64_t radix_tile();            // keys per radix block
uint64_t scan_tile();             // elements per scan block
void scan_u32_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint64_t* n_dev, uint32_t* tmp,
                  uint32_t* total, hipStream_t s);
void scan_u32_u64(const uint32_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, uint64_t* tmp,
                  uint64_t* total, hipStream_t s);
void scan_u64_u64(const uint64_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, uint64_t* tmp,
                  uint64_t* total, hipStream_t s);
int sort_u32_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                 int lo_bit, int hi_bit, const RadixTmp& tmp, hipStream_t s);

// ---- tick buffers handed to the launchers ----------------------------------
struct TickBufs {
    const gw_op* ops;
    uint32_t m;               // ops in the stream
    uint32_t cap;             // total slots
    uint32_t ncells;
    int32_t *last_pos, *last_aoi, *last_leave;
    uint32_t* flags;
    float4* pos;
    AoiEnt* aoi;
    uint8_t* is_mover;
    LstMeta* lst;
    uint32_t* log_cnt;        // [cap] pending log entries per slot
    uint32_t* logs;           // [cap * LOGCAP]
    const SpaceP* sp;
    uint32_t* pool;
    uint64_t pool_cap;
    DevStats* st;
    // grid
    uint32_t* keys;           // [cap]
    uint32_t* cell_cnt;       // [ncells+1]
    uint32_t* cell_start;     // [ncells+1]
    uint32_t* cursor;         // [ncells]
    SortEnt* se;              // [cap]
    uint32_t* pflag;          // [max(cap, m)]
    uint64_t* pre;            // [max(cap, m)]
    uint64_t* fpre;           // [cap] prefix of affected-watcher flags
    // movers
    uint32_t* movers;         // [m] slots, cell order then leavers
    uint64_t* bpk;            // [m] cand | old<<32
    uint64_t* tpk;            // [m] tierS | tierB<<32
    uint64_t* reg_pk;         // [m] exclusive scan of bpk
    uint64_t* tier_pre;       // [m] exclusive scan of tpk
    uint32_t* list_s;         // [m] mover indices of tier S
    uint32_t* list_b;         // [m] tier B
    uint32_t* list_c;         // [m] tier C
    uint64_t* c_temp_off;     // [m] tier C scratch offset (u32 words)
    uint32_t* c_temp;         // tier C scratch
    uint64_t c_temp_cap;
    uint32_t* own;            // own events (targets): [sum cand+old]
    uint64_t* mir;            // mirror events: [sum cand+old]
    uint32_t* mir_cnt;        // [m]
    // canonical events
    unsigned long long* cnt64;  // [cap] enters | leaves<<32 per watcher (zero between ticks)
    uint64_t* off64;          // [cap+1]
    gw_event* enter;
    gw_event* leave;
    uint64_t enter_cap, leave_cap;
    uint32_t* affected;       // [cap]
    uint32_t* bigseg;         // [cap]
    uint64_t* bigseg_off;     // [cap]
    uint32_t* bigseg_temp;
    uint64_t bigseg_temp_cap;
    int write_events;
};

// ---- launchers (kernels.hip) ------------------------------------------------
void tick_ops(const TickBufs& b, hipStream_t s);
void tick_grid(const TickBufs& b, uint64_t* scan_tmp64, uint32_t* scan_tmp32, hipStream_t s);
void tick_movers(const TickBufs& b, uint64_t* scan_tmp64, hipStream_t s);
void tick_bounds(const TickBufs& b, uint64_t* scan_tmp64, hipStream_t s);
void tick_diff(const TickBufs& b, uint64_t n_s, uint64_t n_b, uint64_t n_c, hipStream_t s);
void tick_events(const TickBufs& b, uint64_t n_movers, uint64_t* scan_tmp64, hipStream_t s);
void tick_nonmovers(const TickBufs& b, uint64_t n_affected, uint64_t n_big, uint64_t n_movers, hipStream_t s,
                    bool fuse_sort);
void tick_reset(const TickBufs& b, uint64_t n_movers, hipStream_t s);
void tick_materialize_movers(const TickBufs& b, uint64_t n, bool all, hipStream_t s);
void launch_materialize_slots(LstMeta* lst, uint32_t* pool, uint64_t pool_cap, DevStats* st, uint32_t* log_cnt,
                              uint32_t* logs, const uint32_t* slots, const uint64_t* n_dev, uint64_t n_max,
                              hipStream_t s);
void stats_reduce(DevStats* st, hipStream_t s);

void launch_pool_compact(const LstMeta* lst_in, const uint64_t* new_off, uint32_t cap, const uint32_t* pool_old,
                         uint32_t* pool_new, LstMeta* lst_out, hipStream_t s);
void launch_cap2(const LstMeta* lst, uint32_t cap, uint32_t* out, hipStream_t s);
void launch_set_clients(const uint32_t* slots, const uint16_t* gates, uint32_t n, uint32_t cap,
                        uint16_t* gate, hipStream_t s);
// sync collect
void launch_flag_mark(const uint32_t* flags, uint32_t cap, uint32_t* mark, hipStream_t s);
void launch_flag_compact(const uint32_t* mark, const uint64_t* pre, uint32_t cap, uint32_t* flagged,
                         hipStream_t s);
void launch_sync_count(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, const uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const LstMeta* lst, const uint32_t* pool,
                       uint32_t* cnt, hipStream_t s);
void launch_sync_write(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const LstMeta* lst, const uint32_t* pool,
                       const float4* pos, const uint64_t* rec_off, gw_sync_record* rec, uint64_t rec_cap,
                       uint32_t* act, DevStats* st, hipStream_t s);
void launch_sync_compact(const uint64_t* nf_dev, uint32_t nf_max, const uint64_t* rec_off, const uint32_t* act,
                         const uint64_t* act_off, const gw_sync_record* in, gw_sync_record* out, hipStream_t s);
void launch_gate_hist(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* hist /*65536*/, hipStream_t s);
void launch_gate_keys(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* keys, uint32_t* vals, hipStream_t s);
void launch_gather_records(const gw_sync_record* in, const uint32_t* idx, const uint64_t* n_dev,
                           uint64_t n_max, gw_sync_record* out, hipStream_t s);
void launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);
void launch_fill_i32(int32_t* p, int32_t v, uint64_t n, hipStream_t s);

}  // namespace gw
