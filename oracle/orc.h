/*
 * orc.h — CPU ORACLE for the GoWorld AOI + entity-sync path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in goworld_amd/ links, loads or calls this
 * code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, as the checker / the timed CPU baseline.
 *
 * PARITY UNPINNED at the go-aoi boundary: the AOI arithmetic lives in the
 * third-party module github.com/xiaonanln/go-aoi v0.2.0 (go.mod:25 of the
 * reference), which is neither vendored in /root/reference nor present in any
 * module cache here, and there is no Go toolchain to run the reference.  The
 * reference holds no AOI/sync tests, golden vectors or fixtures (SURVEY.md
 * 8(c)).  This file restates go-aoi's published XZListAOIManager algorithm
 *  and the goworld glue around it, cross-checks it
 * against an independent brute-force restatement, and pins the known-answer
 * facts the reference source does fix (tests/test_oracle.py).
 *
 * Three relation engines share one state/glue layer:
 *   ORC_XZLIST  - faithful restatement of go-aoi XZListAOIManager: X and Z
 *                 sorted doubly linked lists, markVal counting, adjust()
 *                 firing OnEnterAOI/OnLeaveAOI both directions, sequentially
 *                 per op (the reference's immediate, per-call semantics).
 *   ORC_BRUTE   - sequential, O(N) per op: after each op on A, relation(A,b)
 *                 := inWin_A(b) for every present b (independent of the list
 *                 structure; validates ORC_XZLIST).
 *   ORC_SEQRULE - the batched per-tick contract (DESIGN.md / SURVEY Appendix
 *                 B): one net diff per tick, pair decided by the member with
 *                 the larger last-op seq.  This is the spec the GPU implements.
 */
#ifndef ORC_H
#define ORC_H

#include <stdint.h>
#include "../include/gpuaoi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_XZLIST  0
#define ORC_BRUTE   1
#define ORC_SEQRULE 2

typedef struct orc_space orc_space;

/* One space: aoi distance d (Space.EnableAOI(d), Space.go:91-106), local slots
 * 0..capacity-1. */
orc_space* orc_new(uint32_t capacity, float d, int mode);
void       orc_free(orc_space* s);

/* Initial population equal to sequential Enter() of slots[i] in index order
 * (restore path, Space.go:209-214: relations built, no user-visible events). */
int orc_bulk_enter(orc_space* s, uint32_t n, const uint32_t* slots,
                   const float* x, const float* y, const float* z, const float* yaw,
                   uint8_t sync_flags);

/* Apply one tick of ops (slots are local).  Returns 0 or <0 on invalid
 * sequences (Moved/Leave/Sync on an absent slot, Enter on a present one). */
int orc_tick(orc_space* s, const gw_op* ops, uint32_t n);

/* Net directed events of the last tick, canonical (watcher, target) order. */
void orc_event_counts(const orc_space* s, uint64_t* n_enter, uint64_t* n_leave);
void orc_events_copy(const orc_space* s, gw_event* enter, gw_event* leave);
/* Raw callback counts of the last tick (sequential modes; 0 for SEQRULE). */
void orc_raw_counts(const orc_space* s, uint64_t* raw_enter, uint64_t* raw_leave,
                    uint64_t* create_msgs, uint64_t* destroy_msgs);

/* Clients: gate 0 = no client. */
void orc_set_client(orc_space* s, uint32_t slot, uint16_t gate);

/* CollectEntitySyncInfos (Entity.go:1221-1267): records canonical by
 * (gate(watcher), entity, watcher); flags cleared. */
uint64_t orc_collect(orc_space* s);
void     orc_records_copy(const orc_space* s, gw_sync_record* out);

/* Wire encoding of the collected records (Entity.go:1210-1254,
 * netutil LE): per gate packet "u16 1502, u16 gate, {clientid[16] eid[16]
 * f32 x y z yaw}*".  IDs are GenFixedUUID(be32(slot)) / GenFixedUUID(be32(slot)|1<<31)
 * (uuid.go:48-59).  Packets are concatenated in gate order; returns bytes
 * written (or needed when out == NULL). */
uint64_t orc_encode_wire(const orc_space* s, uint8_t* out);
/* GenFixedUUID of a 4-byte big-endian integer -> 16 chars (uuid.go:48-59). */
void orc_fixed_uuid_u32(uint32_t v, char out16[16]);

/* InterestedIn(slot), ascending.  Returns count; copies min(count,cap). */
uint32_t orc_neighbors(const orc_space* s, uint32_t slot, uint32_t* buf, uint32_t cap);
/* InterestedBy(slot) (glue set; equals InterestedIn in every mode). */
uint32_t orc_interested_by(const orc_space* s, uint32_t slot, uint32_t* buf, uint32_t cap);
uint64_t orc_total_neighbors(const orc_space* s);
int      orc_present(const orc_space* s, uint32_t slot);

/* Exact window test of the reference, for tests: other in [fl(c-d), fl(c+d)]
 * on both axes (go-aoi xzlist Mark bounds). */
int orc_in_window(float cx, float cz, float d, float ox, float oz);
/* client messages of the last tick / AllClients fan-out (SURVEY 8(f) ranks
 * 2-3; orc.c has the reference citations); out NULL returns the count */
uint64_t orc_client_creates(const orc_space* s, gw_sync_record* out);
uint64_t orc_client_destroys(const orc_space* s, gw_event* out);
uint64_t orc_fanout(const orc_space* s, const uint32_t* slots, uint32_t n, uint32_t* out);


#ifdef __cplusplus
}
#endif
#endif
