package gpuaoi

/*
#include <stdlib.h>
#include "gpuaoi.h"
*/
import "C"

import (
	"unsafe"

	"github.com/xiaonanln/goworld/engine/gwlog"
)

// WorldRank is one process's strip of a world space decomposed over GPU
// processes (one per GPU; DESIGN.md §6).  The reference keeps a space inside
// one game process (SpaceManager.go:11-31), so this has no reference call
// site: a deployment that splits one huge space adds it around the same game
// loop.  The halo exchange runs inside the library over RCCL (xGMI).
type WorldRank struct {
	*Context // its ops buffer holds this rank's owned calls of the tick (slot = global entity index)
}

// CommUniqueID is called on rank 0; the bytes go to the other ranks over any
// channel (the dispatcher), then every rank calls NewWorldRank.
func CommUniqueID() []byte {
	buf := make([]byte, C.GW_COMM_ID_BYTES)
	if rc := C.gw_comm_unique_id(unsafe.Pointer(&buf[0])); rc != 0 {
		gwlog.Panicf("gpuaoi: gw_comm_unique_id failed: %d", int(rc))
	}
	return buf
}

// NewWorldRank joins the communicator and creates this rank's strip: rank r
// owns entities with x in [x0 + r*stripW, x0 + (r+1)*stripW) (the outer
// strips extend to infinity) and holds every entity within the halo width of
// it; slots are global entity indices in [0, capacity).
func NewWorldRank(device int, id []byte, ranks, rank int, x0, stripW, d, maxStep float32, capacity uint32,
	minX, minZ, maxX, maxZ float32) *WorldRank {
	c := NewContext(device)
	c.check(C.gw_comm_init(c.ctx, unsafe.Pointer(&id[0]), C.int(ranks), C.int(rank)))
	geom := C.gw_world_geom{x0: C.float(x0), strip_w: C.float(stripW), aoi_dist: C.float(d),
		max_step: C.float(maxStep), ranks: C.uint32_t(ranks), rank: C.uint32_t(rank)}
	bounds := [4]C.float{C.float(minX), C.float(minZ), C.float(maxX), C.float(maxZ)}
	var sid C.uint32_t
	c.check(C.gw_world_create(c.ctx, &geom, C.uint32_t(capacity), &bounds[0], &sid))
	return &WorldRank{Context: c}
}

// Op buffers this rank's owned call of the tick: kind GW_OP_*, the global
// entity index, the new position (Enter / Moved) and the syncInfoFlag bits.
func (w *WorldRank) Op(kind uint8, entity uint32, x, y, z, yaw float32, flags uint8) {
	w.ops = append(w.ops, C.gw_op{kind: C.uint8_t(kind), sync_flags: C.uint8_t(flags), slot: C.uint32_t(entity),
		x: C.float(x), y: C.float(y), z: C.float(z), yaw: C.float(yaw)})
}

// Flush of a decomposed-world rank: the owned ops (host memory, call order)
// are checked, staged and routed; the row counts and then exactly the rows
// travel to both neighbours (far rows to any rank holding a teleport's end,
// the long-mover lists to everyone); the tick runs on owned ops + received
// rows; events come back for owned watchers only.  onEvent(leave, watcher,
// target) replays them (the caller maps global indices to its entities).
func (w *WorldRank) Flush(onEvent func(leave bool, watcher, target uint32)) {
	if len(w.ops) > 0 {
		w.check(C.gw_world_step_host(w.ctx, &w.ops[0], C.uint32_t(len(w.ops))))
	} else {
		w.check(C.gw_world_step_host(w.ctx, nil, 0)) // still exchanges: neighbours' rows may arrive
	}
	w.ops = w.ops[:0]
	var out C.gw_tick_out
	w.check(C.gw_tick(w.ctx, C.GW_TICK_COPY_TO_HOST, &out))
	if out.n_leave > 0 {
		for _, ev := range unsafe.Slice(out.leave, int(out.n_leave)) {
			onEvent(true, uint32(ev.watcher), uint32(ev.target))
		}
	}
	if out.n_enter > 0 {
		for _, ev := range unsafe.Slice(out.enter, int(out.n_enter)) {
			onEvent(false, uint32(ev.watcher), uint32(ev.target))
		}
	}
}

// Collect sends the records of the owned entities (one packet per gate) and
// checks the world's contract counters, a collective: every rank calls it at
// the same collect.
func (w *WorldRank) Collect(send func(gate uint16, pkt []byte)) {
	w.Context.Collect(send)
	var overflow, conflicts, badOps C.uint64_t
	w.check(C.gw_world_status(w.ctx, &overflow, &conflicts, &badOps)) // summed over the ranks
	if overflow != 0 || conflicts != 0 || badOps != 0 {
		gwlog.Panicf("gpuaoi: world contract broken: %d halo overflows, %d long-move conflicts, %d bad ops",
			uint64(overflow), uint64(conflicts), uint64(badOps))
	}
}
