// Package gpuaoi binds libgpuaoi.so (include/gpuaoi.h, the MI355X AOI and
// entity-sync path) behind go-aoi's aoi.AOIManager, for LiHeng/goworld.
//
// It is dropped into the goworld tree as engine/gpuaoi, with this repository
// vendored as third_party/goworld_amd (the cgo paths below).  The call-site
// edits in engine/entity and components/game are listed in INTEGRATION.md.
// No Go toolchain exists where this package was written: tests/c_harness.c
// makes the same calls in the same order from plain C and is what the
// repository's tests run; gpuaoi_test.go replays the golden fixtures through
// this package once a maintainer has Go (go generate exports them first).
package gpuaoi

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/goworld_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/goworld_amd/goworld_amd/lib -lgpuaoi -Wl,-rpath,${SRCDIR}/../../third_party/goworld_amd/goworld_amd/lib
#include <stdlib.h>
#include "gpuaoi.h"
*/
import "C"

import (
	"runtime"
	"unsafe"

	"github.com/xiaonanln/go-aoi"
	"github.com/xiaonanln/goworld/engine/gwlog"
)

// syncInfoFlag bits (Entity.go:1199-1204, Space.go:196): the entity's own
// client, the clients of the entities interested in it
const (
	SifOwnClient       uint8 = C.GW_SIF_OWN_CLIENT
	SifNeighborClients uint8 = C.GW_SIF_NEIGHBOR_CLIENTS
)

// Callback is implemented by *entity.Entity (Entity.go:227-233);
// aoi.InitAOI(&e.aoi, d, e, e) (Entity.go:210) stores the entity in a.Data.
type Callback interface {
	OnEnterAOI(other *aoi.AOI)
	OnLeaveAOI(other *aoi.AOI)
}

// Context: one per game process and GPU; every space's Manager shares it.
type Context struct {
	ctx      *C.gw_ctx
	ops      []C.gw_op   // this tick's ops of all spaces, in call order
	aoiOf    []*aoi.AOI  // global slot -> AOI
	mgrOf    []*Manager  // global slot -> its space
	lastKind []C.uint8_t // global slot -> kind of its last op this tick
	touched  []uint32    // slots with an op this tick
}

// NewContext opens the library on HIP device `device` (gw_init fails without
// one: there is no CPU fallback).
func NewContext(device int) *Context {
	runtime.LockOSThread() // single game goroutine, GameService.go:89
	var c *C.gw_ctx
	if rc := C.gw_init(C.int(device), &c); rc != 0 {
		gwlog.Panicf("gpuaoi: gw_init(%d) failed: %d", device, int(rc))
	}
	return &Context{ctx: c}
}

// Close releases the context (gw_shutdown).
func (c *Context) Close() {
	if c.ctx != nil {
		C.gw_shutdown(c.ctx)
		c.ctx = nil
	}
}

func (c *Context) check(rc C.int) {
	if rc != 0 {
		gwlog.Panicf("gpuaoi: %s", C.GoString(C.gw_last_error(c.ctx)))
	}
}

// Manager implements aoi.AOIManager for one space (Space.aoiMgr, Space.go:33).
type Manager struct {
	c      *Context
	sid    C.uint32_t // space id (index | generation: a destroyed space's id is refused afterwards)
	d      aoi.Coord
	base   uint32 // the space's slots are [base, base+cap)
	cap    uint32
	slotOf map[*aoi.AOI]uint32 // global slots
	free   []uint32
}

// NewManager replaces aoi.NewXZListAOIManager(d) at Space.go:105.  capacity
// is a first size (the manager grows itself); the bounds size the device grid
// (entities outside them are still exact, only slower).
func (c *Context) NewManager(d aoi.Coord, capacity uint32, minX, minZ, maxX, maxZ float32) *Manager {
	m := &Manager{c: c, d: d, cap: capacity, slotOf: map[*aoi.AOI]uint32{}}
	bounds := [4]C.float{C.float(minX), C.float(minZ), C.float(maxX), C.float(maxZ)}
	var base C.uint32_t
	c.check(C.gw_space_create(c.ctx, C.float(d), C.uint32_t(capacity), &bounds[0], &m.sid, &base))
	m.base = uint32(base)
	m.freeRange(m.base, capacity)
	c.fit(m.base + capacity)
	return m
}

func (m *Manager) freeRange(from, n uint32) {
	for i := n; i > 0; i-- {
		m.free = append(m.free, from+i-1)
	}
}

// fit grows the slot-indexed tables to n slots.
func (c *Context) fit(n uint32) {
	if int(n) > len(c.aoiOf) {
		k := int(n) - len(c.aoiOf)
		c.aoiOf = append(c.aoiOf, make([]*aoi.AOI, k)...)
		c.mgrOf = append(c.mgrOf, make([]*Manager, k)...)
		c.lastKind = append(c.lastKind, make([]C.uint8_t, k)...)
	}
}

// grow doubles the space when its free list runs out: Space.enter has no
// capacity bound (Space.go:179-217).  gw_space_grow extends the range in
// place or moves the space's state to a new range (new_base); then every
// table that holds one of its slots is remapped, including the ops of this
// tick not yet submitted (the library holds none: they are submitted at Flush).
func (m *Manager) grow() {
	c := m.c
	newCap := 2 * m.cap
	var nb C.uint32_t
	c.check(C.gw_space_grow(c.ctx, m.sid, C.uint32_t(newCap), &nb))
	oldBase, newBase := m.base, uint32(nb)
	c.fit(newBase + newCap)
	if newBase != oldBase {
		remap := func(s uint32) uint32 { return s - oldBase + newBase }
		for i := uint32(0); i < m.cap; i++ { // tables: copy then clear the old range
			o, n := oldBase+i, newBase+i
			c.aoiOf[n], c.mgrOf[n], c.lastKind[n] = c.aoiOf[o], c.mgrOf[o], c.lastKind[o]
			c.aoiOf[o], c.mgrOf[o], c.lastKind[o] = nil, nil, 0
		}
		for a, s := range m.slotOf {
			m.slotOf[a] = remap(s)
		}
		for i, s := range m.free {
			m.free[i] = remap(s)
		}
		for i := range c.ops {
			if s := uint32(c.ops[i].slot); s >= oldBase && s < oldBase+m.cap {
				c.ops[i].slot = C.uint32_t(remap(s))
			}
		}
		for i, s := range c.touched {
			if s >= oldBase && s < oldBase+m.cap {
				c.touched[i] = remap(s)
			}
		}
		m.base = newBase
	}
	m.freeRange(m.base+m.cap, newCap-m.cap)
	m.cap = newCap
}

func (m *Manager) push(kind C.uint8_t, a *aoi.AOI, x, y, z, yaw float32, flags C.uint8_t) {
	c := m.c
	slot, ok := m.slotOf[a]
	if !ok {
		if kind != C.GW_OP_ENTER {
			gwlog.Panicf("gpuaoi: %v not in space", a) // go-aoi: nil implData
		}
		if len(m.free) == 0 {
			m.grow()
		}
		slot = m.free[len(m.free)-1]
		m.free = m.free[:len(m.free)-1]
		m.slotOf[a] = slot
		c.aoiOf[slot], c.mgrOf[slot] = a, m
	}
	if c.lastKind[slot] == 0 {
		c.touched = append(c.touched, slot)
	}
	c.lastKind[slot] = kind
	c.ops = append(c.ops, C.gw_op{kind: kind, sync_flags: flags, slot: C.uint32_t(slot),
		x: C.float(x), y: C.float(y), z: C.float(z), yaw: C.float(yaw)})
}

// Enter, Moved, Leave: aoi.AOIManager.  Enter sets both syncInfoFlag bits
// (Space.go:196); Moved the bits of a server-side move (NEIGHBOR, plus OWN
// through MovedFlags when the move did not come from the client,
// Entity.go:1199-1204); Leave keeps both pending bits (Space.leave leaves the
// flag alone, Space.go:219-242).
func (m *Manager) Enter(a *aoi.AOI, x, z aoi.Coord) {
	m.push(C.GW_OP_ENTER, a, float32(x), 0, float32(z), 0, C.uint8_t(SifOwnClient|SifNeighborClients))
}
func (m *Manager) Moved(a *aoi.AOI, x, z aoi.Coord) {
	m.MovedFlags(a, x, z, SifNeighborClients)
}

// MovedFlags is Moved with the mover's syncInfoFlag bits of this call (edit 2).
func (m *Manager) MovedFlags(a *aoi.AOI, x, z aoi.Coord, flags uint8) {
	m.push(C.GW_OP_MOVED, a, float32(x), 0, float32(z), 0, C.uint8_t(flags))
}
func (m *Manager) Leave(a *aoi.AOI) { m.LeaveKeep(a, SifOwnClient|SifNeighborClients) }

// LeaveKeep is Leave with the mask of pending syncInfoFlag bits the entity
// keeps (0 when it is destroyed or enters another AOI space: Entity.go:136-157).
func (m *Manager) LeaveKeep(a *aoi.AOI, keep uint8) { m.push(C.GW_OP_LEAVE, a, 0, 0, 0, 0, C.uint8_t(keep)) }

// Sync is Entity.SetYaw / a position-yaw update without an AOI move
// (Entity.go:1284-1290): the payload and the flag bits only.
func (m *Manager) Sync(a *aoi.AOI, x, y, z, yaw float32, flags uint8) {
	m.push(C.GW_OP_SYNC, a, x, y, z, yaw, C.uint8_t(flags))
}

// EnterTyped is Enter with the entity type's AOI distance (edit 1b): the
// reference gives it to aoi.InitAOI (Entity.go:210, EntityManager.go:55-63)
// and the space uses its own (Space.go:105); XZList only reads the space's,
// so the two must agree for the results to be go-aoi's (SURVEY App. A).
func (m *Manager) EnterTyped(a *aoi.AOI, x, z, typeDist aoi.Coord) {
	if typeDist != m.d {
		gwlog.Panicf("gpuaoi: entity type AOI distance %v != space AOI distance %v", typeDist, m.d)
	}
	m.Enter(a, x, z)
}

// Slot is the global slot of a in this space (ids, clients, tests).
func (m *Manager) Slot(a *aoi.AOI) (uint32, bool) {
	s, ok := m.slotOf[a]
	return s, ok
}

// Destroy is Space.OnDestroy -> SpaceManager.delSpace (Space.go:143-151,
// SpaceManager.go:25-27): OnDestroy has destroyed the space's entities (their
// Leave calls are buffered), so the tick is flushed (their leave callbacks
// fire, as inside each Leave upstream), then the library checks on the device
// that the space is empty and releases its slot and cell ranges; the id is
// refused from then on (its generation changed).
func (m *Manager) Destroy() {
	c := m.c
	c.Flush()
	if len(m.slotOf) != 0 {
		gwlog.Panicf("gpuaoi: space destroyed with %d entities in it", len(m.slotOf))
	}
	c.check(C.gw_space_destroy(c.ctx, m.sid))
	for i := uint32(0); i < m.cap; i++ {
		c.aoiOf[m.base+i], c.mgrOf[m.base+i], c.lastKind[m.base+i] = nil, nil, 0
	}
	m.free, m.c = nil, nil
}

// Flush is called once per game tick for the whole process (edit 3): one
// submit, one tick, the canonical events of every space, then slot reclaim.
func (c *Context) Flush() {
	if len(c.ops) > 0 {
		c.check(C.gw_submit(c.ctx, &c.ops[0], C.uint32_t(len(c.ops))))
		c.ops = c.ops[:0]
	}
	var out C.gw_tick_out
	c.check(C.gw_tick(c.ctx, C.GW_TICK_COPY_TO_HOST, &out))
	c.replay(&out)
	// a slot whose last op this tick was Leave is free again (its leave events are delivered)
	for _, s := range c.touched {
		if c.lastKind[s] == C.GW_OP_LEAVE {
			m := c.mgrOf[s]
			delete(m.slotOf, c.aoiOf[s])
			c.aoiOf[s], c.mgrOf[s] = nil, nil
			m.free = append(m.free, s)
		}
		c.lastKind[s] = 0
	}
	c.touched = c.touched[:0]
}

// replay fires the tick's callbacks: leaves first, as go-aoi's adjust does.
func (c *Context) replay(out *C.gw_tick_out) {
	if out.n_leave > 0 {
		for _, ev := range unsafe.Slice(out.leave, int(out.n_leave)) {
			c.aoiOf[ev.watcher].Data.(Callback).OnLeaveAOI(c.aoiOf[ev.target])
		}
	}
	if out.n_enter > 0 {
		for _, ev := range unsafe.Slice(out.enter, int(out.n_enter)) {
			c.aoiOf[ev.watcher].Data.(Callback).OnEnterAOI(c.aoiOf[ev.target])
		}
	}
}

// SetIDs registers a slot's entity id, its client id and gate (entity
// creation / client attach, Entity.go:210, GameClient.go:14-27); gate 0 = no client.
func (c *Context) SetIDs(slot uint32, eid, clientid [16]byte, gate uint16) {
	s := C.uint32_t(slot)
	c.check(C.gw_set_entity_ids(c.ctx, &s, unsafe.Pointer(&eid[0]), 1))
	c.check(C.gw_set_client_ids(c.ctx, &s, unsafe.Pointer(&clientid[0]), 1))
	g := C.uint16_t(gate)
	c.check(C.gw_set_clients(c.ctx, &s, &g, 1))
}

// SetClient attaches (gate > 0) or detaches (gate 0) a slot's client (GameClient.go:14-27).
func (c *Context) SetClient(slot uint32, gate uint16) {
	s, g := C.uint32_t(slot), C.uint16_t(gate)
	c.check(C.gw_set_clients(c.ctx, &s, &g, 1))
}

// ClientSync is HandleSyncPositionYawFromClient (GameService.go:395-407): the
// packet's payload after the msgtype, n records of eid[16] x y z yaw, decoded
// into Moved ops on the device side; it returns the records left to the
// caller (entities outside AOI spaces: the reference path handles them).
func (c *Context) ClientSync(payload []byte) (toCaller uint32) {
	var applied, left C.uint32_t
	n := C.uint32_t(len(payload) / 32)
	if n > 0 {
		c.check(C.gw_submit_client_sync(c.ctx, unsafe.Pointer(&payload[0]), n, &applied, &left))
	}
	return uint32(left)
}

// Collect is CollectEntitySyncInfos (Entity.go:1221-1267): the records of
// every flagged entity, encoded as one packet per gate on the device
// (dispatchercluster.SelectByGateID(gate).SendPacket(pkt) in the reference).
func (c *Context) Collect(send func(gate uint16, pkt []byte)) {
	var so C.gw_sync_out
	c.check(C.gw_sync_collect(c.ctx, 0, &so))
	var wo C.gw_wire_out
	c.check(C.gw_sync_encode_wire(c.ctx, C.GW_WIRE_COPY_TO_HOST, &wo))
	if wo.n_packets == 0 {
		return
	}
	bytes := unsafe.Slice((*byte)(unsafe.Pointer(wo.bytes)), int(wo.n_bytes))
	gates := unsafe.Slice(wo.gate, int(wo.n_packets))
	offs := unsafe.Slice(wo.off, int(wo.n_packets)+1)
	for k, g := range gates {
		pkt := make([]byte, int(offs[k+1]-offs[k]))
		copy(pkt, bytes[offs[k]:offs[k+1]])
		send(uint16(g), pkt)
	}
}

// ClientEvents gives the create / destroy client messages of the last tick's
// events in bulk (edit 6: Entity.interest / uninterest send them one by one,
// Entity.go:236-246, GameClient.go:37-59); creates carry the target's
// position and yaw.  Both streams come grouped by gate and client.
func (c *Context) ClientEvents(create func(watcher, target uint32, x, y, z, yaw float32),
	destroy func(watcher, target uint32)) {
	var cr, de C.gw_msg_out
	c.check(C.gw_client_events(c.ctx, C.GW_MSG_COPY_TO_HOST, &cr, &de))
	if cr.n_rec > 0 {
		for _, r := range unsafe.Slice((*C.gw_sync_record)(cr.rec), int(cr.n_rec)) {
			create(uint32(r.watcher), uint32(r.entity), float32(r.x), float32(r.y), float32(r.z), float32(r.yaw))
		}
	}
	if de.n_rec > 0 {
		for _, e := range unsafe.Slice((*C.gw_event)(de.rec), int(de.n_rec)) {
			destroy(uint32(e.watcher), uint32(e.target))
		}
	}
}

// Fanout delivers CallAllClients calls batched per tick (Entity.go:743-749,
// 814-917): call k was made on entity slots[k]; deliver(watcher, entity, k)
// runs once per client that receives it (the caller's own client first, then
// every InterestedBy client), grouped by gate and client.
func (c *Context) Fanout(slots []uint32, deliver func(watcher, entity, call uint32)) {
	if len(slots) == 0 {
		return
	}
	var fo C.gw_msg_out
	c.check(C.gw_fanout(c.ctx, (*C.uint32_t)(unsafe.Pointer(&slots[0])), C.uint32_t(len(slots)),
		C.GW_MSG_COPY_TO_HOST, &fo))
	if fo.n_rec > 0 {
		for _, d := range unsafe.Slice((*C.gw_fanout_rec)(fo.rec), int(fo.n_rec)) {
			deliver(uint32(d.watcher), uint32(d.entity), uint32(d.item))
		}
	}
}
