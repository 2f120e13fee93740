/*
 * gpuaoi.h — C ABI of the MI355X-native GoWorld AOI + entity-sync hot path.
 *
 * This is the drop-in boundary.  A Go shim package (engine/gpuaoi, source in
 * INTEGRATION.md) binds it through cgo; the Python test/bench layer binds it
 * through ctypes.  Plain C types only: no torch, no C++ types, no callbacks.
 *
 * What each entry point replaces in the reference (paths relative to the
 * LiHeng/goworld tree; go-aoi v0.2.0 is the external module named in go.mod:25):
 *
 *   gw_space_create  <- Space.EnableAOI -> aoi.NewXZListAOIManager(d)
 *                       (engine/entity/Space.go:91-106; manager stored in
 *                        Space.aoiMgr, Space.go:33)
 *   gw_submit        <- aoiMgr.Enter / aoiMgr.Moved / aoiMgr.Leave
 *                       (Space.go:201-203, 211-213, 233-235, 250) plus the
 *                       syncInfoFlag updates of Space.go:196,
 *                       Entity.go:1189-1205 (setPositionYaw) and
 *                       Entity.go:1284-1290 (SetYaw)
 *   gw_tick          <- the OnEnterAOI/OnLeaveAOI callbacks go-aoi fires inside
 *                       each call (Entity.go:227-246), batched per tick and
 *                       returned as canonical net event streams
 *   gw_neighbors     <- Entity.InterestedIn / InterestedBy (Entity.go:53-54;
 *                       both sets are equal because go-aoi fires both
 *                       directions of every enter/leave)
 *   gw_sync_collect  <- entity.CollectEntitySyncInfos (Entity.go:1221-1267),
 *                       called from GameService.serveRoutine (GameService.go:186)
 *   gw_set_clients   <- GameClient attach/detach (Entity.client, GameClient.go:14-27)
 *
 * Conventions
 *   - Every function returns 0 on success and a negative GW_E* code on error;
 *     gw_last_error() gives the message.  Nothing throws or longjmps across the
 *     ABI.  The Go shim turns errors into gwlog.Panicf, as the reference panics
 *     on misuse (Space.go:92-102, 184-186, 220-222).
 *   - Slots are GLOBAL per context: a space owns slots
 *     [slot_base, slot_base + capacity) returned by gw_space_create (or
 *     gw_space_grow, which may move them).  Events and sync records carry
 *     global slots, in canonical order over global slots.  Ranges are handed
 *     out first-fit (a destroyed space's range is reused), so without destroys
 *     or moves this is (space, local slot) order.
 *   - One host thread per context; not re-entrant (the reference calls AOI only
 *     from the single game goroutine, GameService.go:89-189).
 *   - Output pointers in gw_tick_out / gw_sync_out are owned by the library and
 *     stay valid until the next gw_tick / gw_sync_collect on the same context.
 *   - Coordinates must be finite.  Only X and Z take part in AOI (Space.go:202,
 *     250); Y and yaw only travel in sync records.
 */
#ifndef GPUAOI_H
#define GPUAOI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define GW_OK          0
#define GW_EINVAL     -1   /* bad argument / misuse (reference would panic)   */
#define GW_ESTATE     -2   /* op sequence invalid for the entity's state       */
#define GW_ENOMEM     -3   /* device or host allocation failed                 */
#define GW_EDEVICE    -4   /* HIP runtime / kernel error                       */
#define GW_ERANGE     -5   /* slot or space id out of range                    */

/* ---- ops ---------------------------------------------------------------- */
#define GW_OP_NOP     0    /* ignored (padding of fixed-size device buffers)   */
#define GW_OP_ENTER   1    /* aoiMgr.Enter(&e.aoi, x, z)      (Space.go:202)   */
#define GW_OP_MOVED   2    /* aoiMgr.Moved(&e.aoi, x, z)      (Space.go:250)   */
#define GW_OP_LEAVE   3    /* aoiMgr.Leave(&e.aoi)            (Space.go:234)   */
#define GW_OP_SYNC    4    /* SetYaw: sync state only, no AOI adjust
                              (Entity.go:1284-1290)                            */

/* syncInfoFlag bits (Entity.go:91-96) */
#define GW_SIF_OWN_CLIENT        1u
#define GW_SIF_NEIGHBOR_CLIENTS  2u

/* One AOI/sync operation, 24 bytes.  Submission order == reference call order
 * (the seq number of the batched-parity contract is the index of the op in
 * the tick's concatenated submission stream).  x,y,z,yaw are the entity's
 * Position and yaw after the op (for LEAVE they are ignored).  sync_flags is
 * ORed into the entity's syncInfoFlag; for a LEAVE it is the mask of pending
 * bits the entity keeps (see the note before gw_space_restore). */
typedef struct gw_op {
    uint8_t  kind;        /* GW_OP_*                                        */
    uint8_t  sync_flags;  /* GW_SIF_* bits set by this call                  */
    uint16_t reserved;    /* must be 0                                       */
    uint32_t slot;        /* global slot                                     */
    float    x, y, z, yaw;
} gw_op;

/* A directed AOI event: watcher.OnEnterAOI(target) / OnLeaveAOI(target). */
typedef struct gw_event {
    uint32_t watcher;
    uint32_t target;
} gw_event;

/* A compact sync record.  The wire form (Entity.go:1231-1253) is
 * clientid(watcher)[16] eid(entity)[16] f32 x,y,z,yaw, grouped per gate;
 * watcher == entity for the own-client record. */
typedef struct gw_sync_record {
    uint32_t watcher;     /* slot whose client receives the record            */
    uint32_t entity;      /* slot whose position/yaw is synced                */
    float    x, y, z, yaw;
} gw_sync_record;

/* gw_tick flags */
#define GW_TICK_COPY_TO_HOST   1u  /* also copy events into pinned host buffers */
#define GW_TICK_NO_EVENTS      2u  /* update neighbour state only (restore/bulk
                                      path, Space.go:209-214)                   */
#define GW_TICK_DEFER          4u  /* device-resident ops only, no COPY_TO_HOST:
                                     launch the tick and return without a host
                                     sync; out holds only `ops`.  The next call
                                     that needs the results settles it (the
                                     collect's one sync covers it); the outputs
                                     are then read with gw_tick_result */

typedef struct gw_tick_out {
    /* canonical order: sorted by (watcher, target); each directed pair at most
       once per tick (net diff, see DESIGN.md "batched parity contract") */
    const gw_event* enter;        /* host pointer (NULL unless COPY_TO_HOST)   */
    const gw_event* leave;
    const gw_event* enter_dev;    /* device pointers, always valid             */
    const gw_event* leave_dev;
    uint64_t n_enter, n_leave;
    uint64_t ops;                 /* ops consumed                              */
    uint64_t movers;              /* distinct slots with an AOI op (M)         */
    uint64_t pairs_tested;        /* candidate pairs evaluated                 */
    uint64_t nbr_old, nbr_new;    /* A_old / A_new: list entries of movers     */
    uint64_t bytes_alg;           /* SURVEY 8(d) algorithmic bytes of the AOI part */
    double   device_us;           /* device time of the tick (HIP events); only
                                     with GW_TICK_COPY_TO_HOST (0 otherwise: the
                                     tick returns before its last kernels end) */
} gw_tick_out;

/* gw_sync_collect flags */
#define GW_SYNC_COPY_TO_HOST   1u
#define GW_SYNC_BY_CLIENT      2u  /* also group the records per client inside each
                                      gate, as GateService.handleSyncPositionYaw
                                      OnClients does (GateService.go:350-375):
                                      order (gate, watcher, entity); client_off
                                      partitions rec, one segment per client
                                      packet MT_SYNC_POSITION_YAW_ON_CLIENTS   */

typedef struct gw_sync_out {
    /* Deterministic order.  Default: grouped by gate(watcher) (gate_off; each
     * gate's packet is one slice), inside a gate by entity ascending; an
     * entity's own-client record first, then its neighbours' records in the
     * order the window walk visits them, i.e. by (grid cell of the watcher's
     * position, watcher slot) - the reference emits them in Go map order, so
     * any fixed order is equivalent and this one costs no sort.  With
     * GW_SYNC_BY_CLIENT: the canonical (gate(watcher), watcher, entity) order
     * of SURVEY App. B.5, each client's records one contiguous segment
     * (client_off).                                                          */
    const gw_sync_record* rec;      /* host pointer (NULL unless COPY_TO_HOST) */
    const gw_sync_record* rec_dev;  /* device pointer, always valid            */
    uint64_t n_rec;
    const uint64_t* gate_off;       /* host: n_gates+1 offsets into rec, by gate id */
    uint32_t n_gates;               /* max gate id + 1                          */
    uint64_t flagged;               /* entities whose syncInfoFlag was set      */
    uint64_t bytes_alg;
    double   device_us;             /* only with COPY_TO_HOST or BY_CLIENT (0
                                       otherwise: the call returns without
                                       waiting for its last kernels)           */
    /* GW_SYNC_BY_CLIENT only: client segments of rec (the watcher slot of each
     * segment; n_clients+1 offsets).  Host arrays with COPY_TO_HOST.          */
    uint32_t n_clients;
    const uint32_t* client_slot;
    const uint64_t* client_off;
    const uint32_t* client_slot_dev;
    const uint64_t* client_off_dev;
} gw_sync_out;

typedef struct gw_ctx gw_ctx;

/* Context on one HIP device (one process per GPU). */
int  gw_init(int device_id, gw_ctx** out);
void gw_shutdown(gw_ctx* ctx);
const char* gw_last_error(const gw_ctx* ctx);

/* Space.EnableAOI(d): d > 0.  bounds = {minx, minz, maxx, maxz} sizes the
 * uniform grid (NULL = Space.GetSpaceRange default, Space.go:52-54); entities
 * outside the bounds are still exact (clamped cells), only slower. */
int  gw_space_create(gw_ctx* ctx, float aoi_dist, uint32_t capacity,
                     const float* bounds, uint32_t* space_id, uint32_t* slot_base);
/* Space.OnDestroy -> SpaceManager.delSpace (Space.go:143-151,
 * SpaceManager.go:25-27; goworld.go:52-60 creates spaces at run time): the
 * space must hold no entity (checked on the device; its entities Leave and
 * are ticked first, as Space.OnDestroy destroys them); its slot and cell
 * ranges are cleared and reused by later creates, its id too. */
int  gw_space_destroy(gw_ctx* ctx, uint32_t space_id);
/* Space.enter has no capacity bound (Space.go:179-217): grow a space to
 * new_capacity slots.  In place when the slots behind it are free (its slots
 * stay), else its state moves to a new range and *new_base receives the new
 * first slot (slot base + i -> new_base + i; the tick / collect outputs of
 * later calls carry the new slots).  No ops may be pending; a world strip
 * grows in place only. */
int  gw_space_grow(gw_ctx* ctx, uint32_t space_id, uint32_t new_capacity, uint32_t* new_base);

/* Slot / cell accounting of the context (capacity-proportional passes run
 * over total_slots and total_cells). */
typedef struct gw_ctx_info {
    uint32_t total_slots;   /* slot range in use: every live space ends below it */
    uint32_t live_slots;    /* capacity of the live spaces                        */
    uint32_t total_cells, live_cells;
    uint32_t live_spaces;
    uint32_t reserved;
} gw_ctx_info;
int  gw_context_info(gw_ctx* ctx, gw_ctx_info* out);

/* Buffer ops (host memory, validated against the entity state; copied). */
int  gw_submit(gw_ctx* ctx, const gw_op* ops, uint32_t n);
/* Buffer ops already resident in device memory (not validated; the caller
 * guarantees a valid sequence).  The pointer must stay valid until gw_tick. */
int  gw_submit_device(gw_ctx* ctx, const gw_op* dev_ops, uint32_t n);

/* Ops already in device memory with explicit global stamps (one u64 per op,
 * also in device memory): the stamp replaces the op's position in the tick's
 * stream when go-aoi's "which member moved last" is decided.
 * Stamps must grow with the reference call order and exceed every stamp used
 * before; a decomposed world (one space split over processes) uses them so
 * that every process orders the ops of all processes the same way. */
int  gw_submit_device_stamped(gw_ctx* ctx, const gw_op* dev_ops, const uint64_t* dev_stamps, uint32_t n);

/* Ownership x-range of a space in a decomposed world: events are emitted only
 * for watchers, and sync records only for entities, whose x (the position
 * after the tick; before it for an entity that left) lies in [x_lo, x_hi).
 * Entities outside it are ghosts mirrored from the neighbouring processes.
 * Default: the whole line. */
int  gw_space_set_ownership(gw_ctx* ctx, uint32_t space_id, float x_lo, float x_hi);

/* ---- decomposed world (one space split into X-strips over processes) ----
 * A halo row (32 B) is an op with its global stamp.  A destination is a
 * neighbour process: the x-range its local space holds (its strip widened by
 * the halo) and a device buffer of cap_entities * 3 rows.  In halo rows
 * op.reserved bit 0 (GW_ROW_LONG) marks the AOI rows of an entity that moved
 * more than max_step in the tick (a teleport); the ops a caller submits keep
 * reserved = 0. */
#define GW_ROW_LONG 1u
typedef struct gw_halo_row {
    gw_op    op;
    uint64_t stamp;
} gw_halo_row;

typedef struct gw_halo_dst {
    float        x_lo, x_hi;     /* the neighbour holds entities with x in [x_lo, x_hi) */
    gw_halo_row* rows;           /* device memory, cap_entities * 3 rows               */
    uint32_t     cap_entities;
    uint32_t     reserved;
} gw_halo_dst;

/* Owner side, BEFORE submitting the same ops: for this process's owned ops
 * of the tick (device memory, with their global stamps) write, per
 * destination, the rows that bring the neighbour's copy of every affected
 * entity up to date, 3 per entity in this order (NOP rows where not needed):
 *   LEAVE   the entity left the space and re-entered inside the tick;
 *   ENTER / MOVED / LEAVE   the net AOI change relative to [x_lo, x_hi),
 *           with the payload and stamp of the entity's last AOI op;
 *   SYNC    the payload of its last non-Leave op and all sync flags pending
 *           since the last collect.
 * Unused rows are zero (GW_OP_NOP).  Reads the entity state before the
 * tick; no host sync.  Entities beyond a buffer's capacity, moves longer
 * than max_step in x and ops with an invalid slot or kind are counted
 * (gw_halo_status). */
int  gw_route_halo(gw_ctx* ctx, const gw_op* dev_ops, const uint64_t* dev_stamps, uint32_t n,
                   float max_step, const gw_halo_dst* dsts, uint32_t n_dst);

/* Receiver side: rows from a neighbour's gw_route_halo (device memory), part
 * of this tick's op stream like gw_submit_device_stamped ops. */
int  gw_submit_device_rows(gw_ctx* ctx, const gw_halo_row* dev_rows, uint32_t n);

/* Counters accumulated by gw_route_halo since the last call (synchronises,
 * then resets them): overflows, owned entities that moved more than
 * max_step (long moves), ops with an invalid slot or kind. */
int  gw_halo_status(gw_ctx* ctx, uint64_t* overflow, uint64_t* long_moves, uint64_t* bad_ops);

/* (GW_OP_LEAVE: sync_flags is the mask of the entity's pending syncInfoFlag
 * bits it keeps.  Space.leave leaves the flag alone (Space.go:219-242), so an
 * entity that stays in the game in the nil space keeps them (pass 3) and the
 * next collect still sends its own-client record at its last position
 * (CollectEntitySyncInfos scans every entity, Entity.go:1221-1239); pass 0
 * when it is destroyed (Entity.go:136-157) or enters another AOI space, whose
 * Enter flags it anew.) */

/* Restore / bulk load (Space.go:209-214 restoreEntity, EntityManager.go:
 * 556-617 freeze/restore): entities slots[i] enter space
 * space_id at (x, z) exactly as n Enter calls in index order would, without
 * events (the restore path fires none), their syncInfoFlag ORed with
 * sync_flags (GW_SIF_*; Space.enter sets both, Space.go:196).  One upload,
 * one kernel and one grid rebuild instead of n ops and a tick.  No ops may be
 * pending; slots must be absent and distinct (all-or-nothing). */
int  gw_space_restore(gw_ctx* ctx, uint32_t space_id, const uint32_t* slots, const float* x, const float* y,
                      const float* z, const float* yaw, uint32_t n, uint8_t sync_flags);

/* Attach / detach clients: gate 0 = no client (GameClient nil). */
int  gw_set_clients(gw_ctx* ctx, const uint32_t* slots, const uint16_t* gates, uint32_t n);

/* Flush all buffered ops of all spaces: AOI update + canonical net events. */
int  gw_tick(gw_ctx* ctx, uint32_t flags, gw_tick_out* out);

/* Outputs of the last tick (settles a GW_TICK_DEFER tick first). */
int  gw_tick_result(gw_ctx* ctx, gw_tick_out* out);

/* CollectEntitySyncInfos for all spaces of the context; clears the flags. */
int  gw_sync_collect(gw_ctx* ctx, uint32_t flags, gw_sync_out* out);

/* One game tick in one call: the position/yaw updates that reach the spaces
 * during a GameService tick (Entity.SetPosition -> Space.move,
 * GameService.go:183-187 / Entity.go:1185-1187) are submitted, flushed
 * (gw_tick) and followed by the tick's CollectEntitySyncInfos (Entity.go:
 * 1221-1267).  ops_on_device != 0: ops is device memory (gw_submit_device);
 * the tick is then deferred and settled by the collect's single host sync
 * (tick_flags may add GW_TICK_COPY_TO_HOST, which forgoes the deferral).  The
 * same as gw_submit + gw_tick + gw_sync_collect + gw_tick_result, with the
 * device never waiting on the host between the tick and the collect.  On a
 * world strip (gw_world_create) the ops are this rank's owned ops and go
 * through gw_world_step / gw_world_step_host (routing + RCCL exchange) instead
 * of gw_submit, every tick, with or without ops. */
int  gw_step(gw_ctx* ctx, const gw_op* ops, uint32_t n, int ops_on_device, uint32_t tick_flags,
             uint32_t sync_flags, gw_tick_out* tick_out, gw_sync_out* sync_out);

/* gw_step over `ticks` consecutive ticks of a device-resident op log (tick t:
 * n ops at dev_ops + t * stride_ops), outputs left on the device: GameService's
 * tick loop (GameService.go:77-190) replayed from a recorded log, e.g. to catch
 * a server up or to measure the path without a per-tick host-language round
 * trip.  Counters of all ticks are summed into *sum (zeroed first). */
typedef struct gw_replay_sum {
    uint64_t ops, movers, n_enter, n_leave, n_rec, pairs_tested, nbr_old, nbr_new, bytes_alg;
} gw_replay_sum;
int  gw_replay(gw_ctx* ctx, const gw_op* dev_ops, uint32_t n, uint64_t stride_ops, uint32_t ticks,
               uint32_t sync_flags, gw_replay_sum* sum);

/* InterestedIn(slot) == InterestedBy(slot), ascending slots. *n receives the
 * full count even when it exceeds cap. */
int  gw_neighbors(gw_ctx* ctx, uint32_t slot, uint32_t* buf, uint32_t cap, uint32_t* n);

/* Per-stage device timings (HIP events recorded around each stage on the
 * library's stream), for bench.py's roofline.  The stages of successive
 * gw_tick / gw_sync_collect calls are all kept until gw_get_stage_times,
 * which synchronises once and returns per stage name the summed time, bytes
 * and number of calls, then clears them; recording adds no host sync and no
 * query to the calls being timed.  name[i] are static strings. */
#define GW_MAX_STAGES 32
typedef struct gw_stage_times {
    uint32_t n;
    const char* name[GW_MAX_STAGES];
    double   us[GW_MAX_STAGES];          /* summed over the calls               */
    uint64_t bytes_alg[GW_MAX_STAGES];   /* algorithmic bytes, summed           */
    uint32_t calls[GW_MAX_STAGES];       /* recorded instances of the stage     */
} gw_stage_times;
int  gw_set_profiling(gw_ctx* ctx, int enable);   /* 0 off, 1 every stage, 2 the "diff" stage only */
int  gw_get_stage_times(gw_ctx* ctx, gw_stage_times* out);

/* ---- client messages ------------------------------
 * Streams of messages to clients, each grouped by the receiving client's gate
 * (gate_off partitions rec by gate id, n_gates = max gate id + 1) and, inside
 * a gate, ordered by receiving watcher slot: one contiguous run per client, in
 * the order the reference's calls reach that client.  Only watchers with a
 * client receive anything (GameClient methods are no-ops on a nil client,
 * GameClient.go:37-59).  Pointers stay valid until the next call of the same
 * entry point. */
#define GW_MSG_COPY_TO_HOST   1u

typedef struct gw_msg_out {
    const void* rec;              /* host (GW_MSG_COPY_TO_HOST), else NULL      */
    const void* rec_dev;          /* device, always valid                       */
    uint64_t n_rec;
    const uint64_t* gate_off;     /* host: n_gates + 1 offsets into rec         */
    uint32_t n_gates;
    uint64_t bytes_alg;           /* records written (+ inputs read)            */
    double   device_us;
} gw_msg_out;

/* Enter/leave events of the last gw_tick turned into the client messages
 * Entity.interest / uninterest send (Entity.go:236-246):
 *   create:  gw_sync_record {watcher, entity = target, x, y, z, yaw of the
 *            target} = GameClient.sendCreateEntity(target, isPlayer=false)
 *            -> MT_CREATE_ENTITY_ON_CLIENT (GameClient.go:37-53,
 *            GoWorldConnection.go:138-153; the host adds type and the
 *            msgpack'd AllClients attributes)
 *   destroy: gw_event {watcher, target} = sendDestroyEntity(target)
 *            -> MT_DESTROY_ENTITY_ON_CLIENT (GameClient.go:55-59)
 * Order: (gate(watcher), watcher, target).  Positions are those at the flush. */
int  gw_client_events(gw_ctx* ctx, uint32_t flags, gw_msg_out* create, gw_msg_out* destroy);

/* AllClients fan-out: n calls, call k on entity slots[k] (Entity.CallAllClients
 * Entity.go:743-749, and every AllClients attribute notification
 * sendMap/ListAttr*ToClients, Entity.go:814-917) reach the entity's own client
 * and the client of every n in InterestedBy (as of the last flush).  Output:
 * gw_fanout_rec {watcher, entity, item = k}, order (gate(watcher), watcher, k),
 * so each client's run lists its calls in call order.  Slots must be in range;
 * an entity outside any AOI space reaches only its own client. */
typedef struct gw_fanout_rec {
    uint32_t watcher;     /* slot whose client receives the call                 */
    uint32_t entity;      /* slots[item]                                          */
    uint32_t item;        /* index of the call                                    */
} gw_fanout_rec;
int  gw_fanout(gw_ctx* ctx, const uint32_t* slots, uint32_t n, uint32_t flags, gw_msg_out* out);

/* Total neighbour-list entries held (sum over slots of |InterestedIn|). */
int  gw_total_neighbors(gw_ctx* ctx, uint64_t* out);

/* Device pointer helpers for device-resident benchmarking. */
int  gw_device_alloc(gw_ctx* ctx, size_t bytes, void** dev_ptr);
int  gw_device_free(gw_ctx* ctx, void* dev_ptr);
int  gw_memcpy_h2d(gw_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
int  gw_memcpy_d2h(gw_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);
int  gw_synchronize(gw_ctx* ctx);

/* Run the context's work on a caller's stream (a hipStream_t of the same
 * device, e.g. torch's current stream, so that device-resident ops produced
 * there and results consumed there need no host synchronisation); NULL
 * restores the context's own stream.  Drains the previous stream first.
 * A collect after a big deferred tick also runs passes on a second stream of
 * the context's own, joined back into this one (by an event) before the
 * collect's statistics are published, so its results are ordered on this
 * stream like everything else. */
int  gw_set_stream(gw_ctx* ctx, void* hip_stream);

/* ---- ids, client-sync decode and the wire encode (host boundary rows) -----
 * EntityID and ClientID are 16-byte strings (engine/common/types.go:9;
 * uuid/uuid.go:27-59).  The context keeps the entity id and the client id of
 * each slot, a host table entity id -> slot for the decode, and the entity's
 * SetClientSyncing flag (Entity.go:437-440). */
#define GW_ID_BYTES 16
int  gw_set_entity_ids(gw_ctx* ctx, const uint32_t* slots, const void* ids /* n*16 */, uint32_t n);
int  gw_clear_entity_ids(gw_ctx* ctx, const uint32_t* slots, uint32_t n);    /* entity destroyed */
int  gw_set_client_ids(gw_ctx* ctx, const uint32_t* slots, const void* ids /* n*16 */, uint32_t n);
int  gw_set_client_syncing(gw_ctx* ctx, const uint32_t* slots, const uint8_t* on, uint32_t n);

/* GameService.HandleSyncPositionYawFromClient (GameService.go:395-407): the
 * payload of one MT_SYNC_POSITION_YAW_FROM_CLIENT packet, n records of
 * eid[16] f32 x y z yaw (little-endian, 32 B each), each in order as
 * entity.OnSyncPositionYawFromClient (EntityManager.go:450-459): a record of
 * an unknown entity is dropped; one whose entity syncs from its client
 * (Entity.go:430-435) becomes setPositionYaw(fromClient=true): a Moved op
 * with syncInfoFlag NEIGHBOR (Entity.go:1189-1205) appended to the tick like
 * gw_submit - if the entity is in an AOI space of this context at that point
 * of the call order; otherwise it is left to the caller (*to_caller counts
 * those: an entity outside AOI spaces keeps the reference path).  *applied:
 * records turned into ops. */
int  gw_submit_client_sync(gw_ctx* ctx, const void* payload, uint32_t n_records, uint32_t* applied,
                           uint32_t* to_caller);

/* The game->gate sync packets of the last gw_sync_collect (Entity.go:1210-1266):
 * per gate with records, u16 MT_SYNC_POSITION_YAW_ON_CLIENTS (1502), u16
 * gateid, then per record clientid(watcher)[16] eid(entity)[16] f32 x y z yaw
 * (48 B, little-endian), records in the collect's order.  Encoded on the
 * device; `bytes` is one buffer holding the packets back to back, packet k of
 * gate gate[k] at [off[k], off[k+1]).  Pointers valid until the next call. */
#define GW_WIRE_COPY_TO_HOST 1u
typedef struct gw_wire_out {
    const uint8_t* bytes;         /* host (GW_WIRE_COPY_TO_HOST), else NULL     */
    const uint8_t* bytes_dev;     /* device, always valid                       */
    uint64_t n_bytes;
    uint32_t n_packets;
    const uint16_t* gate;         /* host: n_packets gate ids                   */
    const uint64_t* off;          /* host: n_packets + 1 byte offsets           */
    double device_us;
} gw_wire_out;
int  gw_sync_encode_wire(gw_ctx* ctx, uint32_t flags, gw_wire_out* out);

/* ---- RCCL communicator (one per context: one process per GPU) -----------
 * The data-path collectives of a decomposed world run inside the library on
 * the context's stream (RCCL over xGMI), so a Go host drives them through the
 * same C ABI.  Rank 0 makes the id, the host distributes it (any channel),
 * every rank calls gw_comm_init (blocking until all have joined). */
#define GW_COMM_ID_BYTES 128
int  gw_comm_unique_id(void* id /* GW_COMM_ID_BYTES */);
int  gw_comm_init(gw_ctx* ctx, const void* id, int nranks, int rank);
int  gw_comm_info(gw_ctx* ctx, int* nranks, int* rank);      /* 0 ranks: no communicator */
/* Loopback communicator: the nranks contexts of ONE process become ranks
 * 0..nranks-1 of a group whose collectives copy between their buffers
 * (hipMemcpyAsync on the contexts' streams) with the semantics of the RCCL
 * path - same calls, same matching, same ordering.  Each context is then
 * driven by its own host thread exactly as a rank process drives its own
 * (gw_world_step / gw_comm_exchange block until the peers' matching calls
 * are issued; a peer that never issues them fails the call after
 * GW_LOOPBACK_TIMEOUT_S seconds, default 120).  For running the multi-rank
 * world sequence on one device; the contexts may share it. */
int  gw_comm_init_local(gw_ctx* const* ctxs, int nranks);

/* One transfer of a grouped point-to-point exchange (bytes, device memory). */
typedef struct gw_xfer {
    int32_t     peer;
    uint32_t    reserved;
    const void* send;  uint64_t send_bytes;   /* 0: nothing to send to peer   */
    void*       recv;  uint64_t recv_bytes;   /* 0: nothing to receive        */
} gw_xfer;
/* ncclGroupStart; ncclSend / ncclRecv per transfer; ncclGroupEnd, on the
 * context's stream (asynchronous; the peer may be this rank itself). */
int  gw_comm_exchange(gw_ctx* ctx, const gw_xfer* x, uint32_t n);
#define GW_RED_SUM 0
#define GW_RED_MAX 1
/* In-place ncclAllReduce of n u64 device words on the context's stream. */
int  gw_comm_allreduce_u64(gw_ctx* ctx, uint64_t* dev, uint32_t n, int op);

/* ---- decomposed world: one space split into X-strips, one per context ----
 * Strip r owns entities with x in [x0 + r*w, x0 + (r+1)*w) (strip 0 and the
 * last one extend to -inf / +inf) and holds, in one local space whose slots
 * are the global entity ids, every entity within h = d + 2*max_step + 1 +
 * 1e-5*(|x0| + ranks*w) of it (owned + ghosts).  Per tick:
 * the owned ops get global stamps 1 + (tick*ranks + rank)*2^26 + i, their net
 * effect is routed to both neighbours as halo rows (gw_route_halo's rows),
 * the row counts and then exactly the rows are exchanged, and the owned ops
 * plus the received rows form the tick's op stream.  Events are emitted only
 * for owned watchers, records only for owned entities. */
typedef struct gw_world_geom {
    float    x0;         /* strip r covers [x0 + r*strip_w, x0 + (r+1)*strip_w)   */
    float    strip_w;    /* strip width                                         */
    float    aoi_dist;   /* d (EnableAOI)                                       */
    float    max_step;   /* max |dx| of a present owned entity per tick         */
    uint32_t ranks, rank;
} gw_world_geom;
/* bounds: the grid of the local space (its held x-range and the world's z). */
int  gw_world_create(gw_ctx* ctx, const gw_world_geom* geom, uint32_t capacity, const float* bounds,
                     uint32_t* space_id);
/* One tick with the exchange over the context's communicator (ranks > 1
 * needs gw_comm_init): route, count exchange, one host sync, exact row
 * exchange, queue (then gw_tick / gw_sync_collect as usual).  dev_ops: this
 * rank's owned ops of the tick in call order, valid until the tick. */
int  gw_world_step(gw_ctx* ctx, const gw_op* dev_ops, uint32_t n);
/* The same tick with the exchange done by the caller (another transport):
 * gw_world_route writes the rows (one host sync) and returns the rows per
 * neighbour (entities * 3 rows; send[0] left, send[1] right, NULL if none);
 * the caller sends them, receives the neighbours' rows and calls
 * gw_world_submit with them (device memory, valid until the tick). */
int  gw_world_route(gw_ctx* ctx, const gw_op* dev_ops, uint32_t n, const gw_halo_row* send[2],
                    uint32_t send_rows[2]);
int  gw_world_submit(gw_ctx* ctx, const gw_halo_row* const recv[2], const uint32_t recv_rows[2]);
/* Host ops (the Go caller's Space.enter / leave / move calls of the tick on
 * the entities this rank owns, host memory, call order; Space.go:179-252,
 * Entity.go:1185-1205): checked for what needs no entity state (kind,
 * reserved = 0, entity id inside the world's id range, finite x/z for
 * Enter/Moved; presence is the owner's device state), copied through a
 * pinned buffer into a device buffer the library owns; *dev_ops stays valid
 * until the tick that consumes it.  Then gw_world_step or gw_world_route as
 * with device ops.  gw_world_step_host = stage + gw_world_step. */
int  gw_world_stage_ops(gw_ctx* ctx, const gw_op* ops, uint32_t n, const gw_op** dev_ops);
int  gw_world_step_host(gw_ctx* ctx, const gw_op* ops, uint32_t n);
/* Long moves (an owned entity moving more than max_step in x in one tick, e.g.
 * SetPosition far away, Entity.go:1185-1187): besides its
 * neighbours, every rank whose held range contains the entity's old or new
 * position gets its rows, and the owner gets a LEAVE row for its own copy
 * when the entity left the owner's held range.  gw_world_step exchanges them
 * itself (an all-gather of the per-rank counts when there are >= 3 ranks,
 * then the rows with the neighbours' in one grouped round).  On the caller's
 * transport: after gw_world_route, gw_world_far gives these rows grouped by
 * destination rank (counts[q] entities = 3 rows each, rank q's at the sum of
 * the counts before q; counts has `ranks` entries, this rank's own LEAVE rows
 * under its own rank); the caller delivers them and every rank queues what it
 * received (its own included) with gw_world_submit_far after gw_world_submit
 * (device memory, valid until the tick).  Events of a long mover's pairs with
 * entities that are not long movers are emitted by the owner of the other
 * member; pairs of two long movers (a group teleport) by the owner of the
 * watcher's new position, from the long lists (gw_world_longs below). */
int  gw_world_far(gw_ctx* ctx, const gw_halo_row** rows, const uint32_t** counts);
int  gw_world_submit_far(gw_ctx* ctx, const gw_halo_row* rows, uint32_t n_rows);
/* Group teleports (Entity.SetPosition of several related entities in one
 * tick, Entity.go:1185; enterLocalSpace moves entities together, Entity.go:
 * 975-998): a pair of long movers may be related before the tick on one rank
 * and after it on another, so no rank holds both ends of the pair.  Every long
 * mover is therefore also listed once, by its owner, with its state before
 * and after the tick (position and the stamp of its last AOI op); all ranks
 * receive every rank's list, and the owner of each long mover's new position
 * evaluates its pairs with the other long movers from the lists (the seq rule
 * of DESIGN.md §2 needs only those positions and stamps) and emits its events.
 * gw_world_step exchanges the lists itself.  On the caller's transport: after
 * gw_world_route, gw_world_longs gives this rank's list (device memory,
 * *n entries); the caller all-gathers the lists and queues the concatenation
 * of all ranks' lists (its own included, any order) with gw_world_submit_longs
 * after gw_world_submit (device memory, valid until the tick). */
typedef struct gw_long_move {
    uint32_t slot;                    /* global entity id                       */
    uint32_t reserved[3];
    float    old_x, old_z, new_x, new_z;
    uint64_t old_stamp, new_stamp;    /* stamps of its last AOI op before / after */
} gw_long_move;
int  gw_world_longs(gw_ctx* ctx, const gw_long_move** rows, uint32_t* n);
int  gw_world_submit_longs(gw_ctx* ctx, const gw_long_move* rows, uint32_t n);
/* Contract counters since the last call, summed over ranks when a
 * communicator exists: halo overflows (0 by construction), long-move
 * conflicts (pairs of long movers the lists did not cover: 0 unless a rank's
 * long list was not queued for its tick), ops with an invalid slot or kind. */
int  gw_world_status(gw_ctx* ctx, uint64_t* overflow, uint64_t* conflicts, uint64_t* bad_ops);

/* ABI version (bumped on layout changes). */
#define GW_ABI_VERSION 15
int  gw_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GPUAOI_H */
