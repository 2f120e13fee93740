// gw_internal.hpp — device data layout shared by kernels.hip and capi.cpp.
//
// Per context (one HIP device) the state of all spaces lives in one set of
// slot-indexed SoA arrays in HBM ("shard"); a space owns a contiguous slot
// range and a contiguous range of uniform-grid cells, so one launch ticks
// every space of the device at once (BASELINE config #4: 10k spaces).
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

// Per-space parameters (32 B).  Cells are squares of side cs = 1/inv_cs >= d
// (DESIGN.md): a window spans at most 3x3 cells.  Any cell function that is
// monotone in x and z keeps the search exact, whatever the float rounding.
struct alignas(16) SpaceP {
    float d;
    float x0, z0, inv_cs;
    int32_t W, H;
    uint32_t cell_base;
    uint32_t alive;
};

// Device-side counters of one tick / collect (read back once per call).
struct DevStats {
    unsigned long long bound_total;   // sum over movers of 2*(candidates + |old list|)
    unsigned long long a_old;         // sum over movers of |old list|
    unsigned long long a_new;         // sum over movers of |new list|
    unsigned long long pairs_tested;
    unsigned long long ev_count;      // events emitted into the scratch buffer
    unsigned long long ev_overflow;
    unsigned long long total_entries; // sum over slots of |list|
    unsigned long long pool_top;      // bump pointer of the neighbour pool (entries)
    unsigned long long pool_overflow;
    unsigned long long movers;        // distinct AOI-op slots
    unsigned long long n_present;     // entities in the grid
    unsigned long long scan_total;    // generic scan total
    unsigned long long ev_scan_total; // packed (segments<<32 | enters)
    unsigned long long flagged;       // sync: flagged entities
    unsigned long long rec_total;     // sync: records
    unsigned long long bad_ops;       // ops with slot out of range
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
int sort_u64(uint64_t* k0, uint64_t* k1, uint64_t n_max, const uint64_t* n_dev, int lo_bit, int hi_bit,
             const RadixTmp& tmp, hipStream_t s);

// ---- kernel launchers (kernels.hip) ---------------------------------------
void launch_ops(const gw_op* ops, uint32_t m, uint32_t cap, int32_t* last_pos, int32_t* last_aoi,
                int32_t* last_leave, uint32_t* flags, float4* pos, AoiEnt* aoi, uint32_t* is_last,
                DevStats* st, hipStream_t s);
void launch_compact_movers(const gw_op* ops, uint32_t m, const uint32_t* is_last, const uint64_t* pre,
                           uint32_t* movers, hipStream_t s);
void launch_cell_keys(const AoiEnt* aoi, const SpaceP* sp, uint32_t cap, uint32_t ncells,
                      uint32_t* keys, uint32_t* vals, uint32_t* cell_cnt, hipStream_t s);
void launch_gather_sorted(const uint32_t* vals, const AoiEnt* aoi, const uint32_t* n_present_dev,
                          uint32_t cap, SortEnt* se, DevStats* st, hipStream_t s);
void launch_bounds(const uint32_t* movers, const uint64_t* n_movers_dev, uint32_t m_max,
                   const AoiEnt* aoi, const SpaceP* sp, const uint32_t* cell_start,
                   const uint32_t* lst_cnt, DevStats* st, hipStream_t s);
void launch_diff(const uint32_t* movers, const uint64_t* n_movers_dev, uint32_t m_max,
                 const AoiEnt* aoi, const SpaceP* sp, const uint32_t* cell_start, const SortEnt* se,
                 const uint32_t* lst_off, const uint32_t* lst_cnt, const uint32_t* pool,
                 uint64_t* ev, uint64_t ev_cap, int sb, DevStats* st, hipStream_t s);
void launch_ev_flags(const uint64_t* ev, const uint64_t* n_ev_dev, uint64_t n_max, int sb,
                     uint64_t* packed, hipStream_t s);
void launch_ev_split(const uint64_t* ev, const uint64_t* n_ev_dev, uint64_t n_max, int sb,
                     const uint64_t* packed_excl, gw_event* enter, gw_event* leave, uint32_t* seg_start,
                     int write_events, hipStream_t s);
void launch_list_update(const uint64_t* ev, const uint64_t* packed_excl, const uint32_t* seg_start,
                        const unsigned long long* ev_scan_total, uint64_t seg_max, int sb,
                        const AoiEnt* aoi, uint32_t* lst_off, uint32_t* lst_cnt, const uint32_t* pool_old,
                        uint32_t* pool_new, uint64_t pool_cap, DevStats* st, hipStream_t s);
void launch_tick_reset(const gw_op* ops, uint32_t m, uint32_t cap, int32_t* last_pos, int32_t* last_aoi,
                       int32_t* last_leave, AoiEnt* aoi, hipStream_t s);
void launch_pool_compact(const uint32_t* lst_off, const uint32_t* lst_cnt, const uint64_t* new_off,
                         uint32_t cap, const uint32_t* pool_old, uint32_t* pool_new, uint32_t* lst_off_out,
                         hipStream_t s);
void launch_set_clients(const uint32_t* slots, const uint16_t* gates, uint32_t n, uint32_t cap,
                        uint16_t* gate, hipStream_t s);
// sync collect
void launch_flag_mark(const uint32_t* flags, uint32_t cap, uint32_t* mark, hipStream_t s);
void launch_flag_compact(const uint32_t* mark, const uint64_t* pre, uint32_t cap, uint32_t* flagged,
                         hipStream_t s);
void launch_sync_count(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, const uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const uint32_t* lst_off,
                       const uint32_t* lst_cnt, const uint32_t* pool, uint32_t* cnt, hipStream_t s);
void launch_sync_write(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const uint32_t* lst_off,
                       const uint32_t* lst_cnt, const uint32_t* pool, const float4* pos,
                       const uint64_t* rec_off, gw_sync_record* rec, uint64_t rec_cap, hipStream_t s);
void launch_gate_hist(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* hist /*65536*/, hipStream_t s);
void launch_gate_keys(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* keys, uint32_t* vals, hipStream_t s);
void launch_gather_records(const gw_sync_record* in, const uint32_t* idx, const uint64_t* n_dev,
                           uint64_t n_max, gw_sync_record* out, hipStream_t s);
void launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);
void launch_fill_i32(int32_t* p, int32_t v, uint64_t n, hipStream_t s);

}  // namespace gw
