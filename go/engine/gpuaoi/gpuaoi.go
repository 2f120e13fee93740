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
	"github.com/xiaonanln/goworld/engine/proto"
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

// SyncInfoSource is implemented by *entity.Entity through a one-line method
// (INTEGRATION.md edit 2): the record payload CollectEntitySyncInfos reads,
// e.Position.X/Y/Z and e.yaw (getSyncInfo, Entity.go:1269-1276).  The
// aoi.AOIManager calls carry only x and z, so the Y and yaw of an Enter /
// Moved come from here when the tick's calls are submitted (after
// setPositionYaw has set e.yaw, Entity.go:1189-1205; before the collect,
// which reads the same fields).
type SyncInfoSource interface {
	AOISyncInfo() proto.EntitySyncInfo
}

// entInfo: what the wire records need of an entity (ids and client) and its
// SetClientSyncing flag; applied to whichever slot the entity holds.
type entInfo struct {
	eid, cid [16]byte
	gate     uint16
	syncing  bool
}

type parkRef struct {
	m *Manager
	a *aoi.AOI
}

// Context: one per game process and GPU; every space's Manager shares it.
type Context struct {
	ctx       *C.gw_ctx
	ops       []C.gw_op   // this tick's ops of all spaces not yet submitted, in call order
	resolve   []int       // ops whose y / yaw come from the entity at submit (SyncInfoSource)
	submitted bool        // ops reached the library since the last gw_tick
	aoiOf     []*aoi.AOI  // global slot -> AOI
	mgrOf     []*Manager  // global slot -> its space
	lastKind  []C.uint8_t // global slot -> kind of its last op this tick
	lastKeep  []uint8     // global slot -> keep-mask of its last Leave this tick
	touched   []uint32    // slots with an op this tick
	parked    []parkRef   // left with pending sync bits: freed after the next Collect
	ent       map[*aoi.AOI]*entInfo
	cur       map[*aoi.AOI]*Manager // the space whose slot holds the entity's ids
	idDirty   map[*aoi.AOI]bool     // ids / client / syncing to (re)apply at that slot
	nbuf      []C.uint32_t          // gw_neighbors buffer (Restore)
}

// NewContext opens the library on HIP device `device` (gw_init fails without
// one: there is no CPU fallback).
func NewContext(device int) *Context {
	runtime.LockOSThread() // single game goroutine, GameService.go:89
	var c *C.gw_ctx
	if rc := C.gw_init(C.int(device), &c); rc != 0 {
		gwlog.Panicf("gpuaoi: gw_init(%d) failed: %d", device, int(rc))
	}
	return &Context{ctx: c, ent: map[*aoi.AOI]*entInfo{}, cur: map[*aoi.AOI]*Manager{},
		idDirty: map[*aoi.AOI]bool{}}
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
	slotOf map[*aoi.AOI]uint32 // global slots (live entities and parked ones)
	parked map[*aoi.AOI]bool   // left with pending sync bits, slot kept until the next Collect
	free   []uint32
}

// NewManager replaces aoi.NewXZListAOIManager(d) at Space.go:105.  capacity
// is a first size (the manager grows itself); the bounds size the device grid
// (entities outside them are still exact, only slower).
func (c *Context) NewManager(d aoi.Coord, capacity uint32, minX, minZ, maxX, maxZ float32) *Manager {
	m := &Manager{c: c, d: d, cap: capacity, slotOf: map[*aoi.AOI]uint32{}, parked: map[*aoi.AOI]bool{}}
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
		c.lastKeep = append(c.lastKeep, make([]uint8, k)...)
	}
}

// grow doubles the space when its free list runs out: Space.enter has no
// capacity bound (Space.go:179-217).  gw_space_grow extends the range in
// place or moves the space's state to a new range (new_base); then every
// table that holds one of its slots is remapped, including the ops of this
// tick not yet submitted.  Ops already submitted would pin the range, so
// they are ticked first (gw_space_grow needs none pending).
func (m *Manager) grow() {
	c := m.c
	if c.submitted { // (after a ClientSync this tick): those ops are ticked first, a tick boundary early
		c.Flush()
	}
	newCap := 2 * m.cap
	var nb C.uint32_t
	c.check(C.gw_space_grow(c.ctx, m.sid, C.uint32_t(newCap), &nb))
	oldBase, newBase := m.base, uint32(nb)
	c.fit(newBase + newCap)
	if newBase != oldBase {
		remap := func(s uint32) uint32 { return s - oldBase + newBase }
		for i := uint32(0); i < m.cap; i++ { // tables: copy then clear the old range
			o, n := oldBase+i, newBase+i
			c.aoiOf[n], c.mgrOf[n], c.lastKind[n], c.lastKeep[n] = c.aoiOf[o], c.mgrOf[o], c.lastKind[o], c.lastKeep[o]
			c.aoiOf[o], c.mgrOf[o], c.lastKind[o], c.lastKeep[o] = nil, nil, 0, 0
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

// take gives a its slot for an Enter (or a restore): a new one, or the one it
// left this tick or with pending sync bits since the last Collect - back into
// the same slot, so its pending bits and the Enter's join as the reference's
// single syncInfoFlag does.
func (m *Manager) take(a *aoi.AOI) uint32 {
	c := m.c
	if s, ok := m.slotOf[a]; ok {
		if m.parked[a] {
			delete(m.parked, a)
		} else if c.lastKind[s] != C.GW_OP_LEAVE {
			gwlog.Panicf("gpuaoi: %v entered a space it is in", a) // go-aoi: Enter twice
		}
		c.cur[a], c.idDirty[a] = m, true
		return s
	}
	if len(m.free) == 0 {
		m.grow()
	}
	s := m.free[len(m.free)-1]
	m.free = m.free[:len(m.free)-1]
	m.slotOf[a] = s
	c.aoiOf[s], c.mgrOf[s] = a, m
	c.cur[a], c.idDirty[a] = m, true
	return s
}

// release frees a slot once its leave events are delivered (and, if it kept
// sync bits, once they were collected).
func (m *Manager) release(s uint32, a *aoi.AOI) {
	c := m.c
	delete(m.slotOf, a)
	delete(m.parked, a)
	if c.cur[a] == m {
		delete(c.cur, a)
	}
	c.aoiOf[s], c.mgrOf[s] = nil, nil
	m.free = append(m.free, s)
}

func (m *Manager) push(kind C.uint8_t, a *aoi.AOI, x, y, z, yaw float32, flags C.uint8_t, resolve bool) {
	c := m.c
	var slot uint32
	if kind == C.GW_OP_ENTER {
		slot = m.take(a)
	} else {
		s, ok := m.slotOf[a]
		if !ok || m.parked[a] {
			gwlog.Panicf("gpuaoi: %v not in space", a) // go-aoi: nil implData
		}
		slot = s
	}
	if c.lastKind[slot] == 0 {
		c.touched = append(c.touched, slot)
	}
	c.lastKind[slot] = kind
	if kind == C.GW_OP_LEAVE {
		c.lastKeep[slot] = uint8(flags)
	}
	if resolve {
		c.resolve = append(c.resolve, len(c.ops))
	}
	c.ops = append(c.ops, C.gw_op{kind: kind, sync_flags: flags, slot: C.uint32_t(slot),
		x: C.float(x), y: C.float(y), z: C.float(z), yaw: C.float(yaw)})
}

// Enter, Moved, Leave: aoi.AOIManager.  Enter sets both syncInfoFlag bits
// (Space.go:196); Moved the bits of a server-side move (NEIGHBOR, plus OWN
// through MovedFlags when the move did not come from the client,
// Entity.go:1199-1204); Leave keeps both pending bits (Space.leave leaves the
// flag alone, Space.go:219-242).  The record payload's Y and yaw are the
// entity's (SyncInfoSource) at submit time.
func (m *Manager) Enter(a *aoi.AOI, x, z aoi.Coord) {
	m.push(C.GW_OP_ENTER, a, float32(x), 0, float32(z), 0, C.uint8_t(SifOwnClient|SifNeighborClients), true)
}
func (m *Manager) Moved(a *aoi.AOI, x, z aoi.Coord) {
	m.MovedFlags(a, x, z, SifNeighborClients)
}

// MovedFlags is Moved with the mover's syncInfoFlag bits of this call (edit 2).
func (m *Manager) MovedFlags(a *aoi.AOI, x, z aoi.Coord, flags uint8) {
	m.push(C.GW_OP_MOVED, a, float32(x), 0, float32(z), 0, C.uint8_t(flags), true)
}

// EnterPos and MovedPos take the whole payload from the call site (x, y, z,
// yaw = e.Position and e.yaw after the call), for callers that have it.
func (m *Manager) EnterPos(a *aoi.AOI, x, y, z, yaw float32) {
	m.push(C.GW_OP_ENTER, a, x, y, z, yaw, C.uint8_t(SifOwnClient|SifNeighborClients), false)
}
func (m *Manager) MovedPos(a *aoi.AOI, x, y, z, yaw float32, flags uint8) {
	m.push(C.GW_OP_MOVED, a, x, y, z, yaw, C.uint8_t(flags), false)
}
func (m *Manager) Leave(a *aoi.AOI) { m.LeaveKeep(a, SifOwnClient|SifNeighborClients) }

// LeaveKeep is Leave with the mask of pending syncInfoFlag bits the entity
// keeps (0 when it is destroyed or enters another AOI space: Entity.go:136-157).
// A slot that keeps bits stays the entity's until the next Collect has sent
// its own-client record (CollectEntitySyncInfos scans every entity,
// Entity.go:1221-1239).
func (m *Manager) LeaveKeep(a *aoi.AOI, keep uint8) {
	m.push(C.GW_OP_LEAVE, a, 0, 0, 0, 0, C.uint8_t(keep), false)
}

// Sync is Entity.SetYaw / a position-yaw update without an AOI move
// (Entity.go:1284-1290): the payload and the flag bits only.
func (m *Manager) Sync(a *aoi.AOI, x, y, z, yaw float32, flags uint8) {
	m.push(C.GW_OP_SYNC, a, x, y, z, yaw, C.uint8_t(flags), false)
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

// Slot is the global slot of a in this space (tests).
func (m *Manager) Slot(a *aoi.AOI) (uint32, bool) {
	s, ok := m.slotOf[a]
	return s, ok && !m.parked[a]
}

// RestoreEntry is one entity of a restored space: its Position and yaw from
// the freeze data (restoreEntity, EntityManager.go:246-300).
type RestoreEntry struct {
	A            *aoi.AOI
	X, Y, Z, Yaw float32
}

// Restore is Space.enter(e, pos, isRestore=true) (Space.go:209-214) for a
// whole space at once (RestoreFreezedEntities, EntityManager.go:556-617;
// edit 1): gw_space_restore writes the state of len(ents) Enter calls in
// index order in one upload and one kernel (syncInfoFlag |= OWN | NEIGHBOR,
// Space.go:196).  go-aoi fires OnEnterAOI both ways for every pair inside
// those Enters; their clients are attached only afterwards
// (EntityManager.go:605-613), so no client message goes out and what
// remains is InterestedIn / InterestedBy: the callbacks are fired here from
// the relation the restore left on the device (gw_neighbors), each directed
// pair once.
func (m *Manager) Restore(ents []RestoreEntry) {
	c := m.c
	n := len(ents)
	if n == 0 {
		return
	}
	if len(c.ops) > 0 || c.submitted {
		c.Flush() // gw_space_restore needs no pending ops; earlier calls come first
	}
	for uint32(len(m.free)) < uint32(n) {
		m.grow()
	}
	slots := make([]C.uint32_t, n)
	xs, ys, zs, yaws := make([]C.float, n), make([]C.float, n), make([]C.float, n), make([]C.float, n)
	in := make(map[*aoi.AOI]bool, n)
	for i, e := range ents {
		if in[e.A] {
			gwlog.Panicf("gpuaoi: %v restored twice", e.A)
		}
		in[e.A] = true
		slots[i] = C.uint32_t(m.take(e.A))
		xs[i], ys[i], zs[i], yaws[i] = C.float(e.X), C.float(e.Y), C.float(e.Z), C.float(e.Yaw)
	}
	c.applyIDs()
	c.check(C.gw_space_restore(c.ctx, m.sid, &slots[0], &xs[0], &ys[0], &zs[0], &yaws[0], C.uint32_t(n),
		C.uint8_t(SifOwnClient|SifNeighborClients)))
	for i, e := range ents {
		for _, o := range c.neighbors(uint32(slots[i])) {
			other := c.aoiOf[o]
			e.A.Data.(Callback).OnEnterAOI(other)
			if !in[other] { // the other direction of a pair with an entity already in the space
				other.Data.(Callback).OnEnterAOI(e.A)
			}
		}
	}
}

// neighbors: InterestedIn(slot) == InterestedBy(slot), ascending slots.
func (c *Context) neighbors(slot uint32) []C.uint32_t {
	if len(c.nbuf) == 0 {
		c.nbuf = make([]C.uint32_t, 256)
	}
	for {
		var n C.uint32_t
		c.check(C.gw_neighbors(c.ctx, C.uint32_t(slot), &c.nbuf[0], C.uint32_t(len(c.nbuf)), &n))
		if int(n) <= len(c.nbuf) {
			return c.nbuf[:n]
		}
		c.nbuf = make([]C.uint32_t, 2*int(n))
	}
}

// Destroy is Space.OnDestroy -> SpaceManager.delSpace (Space.go:143-151,
// SpaceManager.go:25-27): OnDestroy has destroyed the space's entities (their
// Leave calls are buffered), so the tick is flushed (their leave callbacks
// fire, as inside each Leave upstream), then the library checks on the device
// that the space is empty and releases its slot and cell ranges; the id is
// refused from then on (its generation changed).  Entities that left it into
// the nil space since the last Collect lose their pending own-client record
// with it (collect first to keep them).
func (m *Manager) Destroy() {
	c := m.c
	c.Flush()
	for a := range m.parked {
		m.release(m.slotOf[a], a)
	}
	if len(m.slotOf) != 0 {
		gwlog.Panicf("gpuaoi: space destroyed with %d entities in it", len(m.slotOf))
	}
	c.check(C.gw_space_destroy(c.ctx, m.sid))
	for i := uint32(0); i < m.cap; i++ {
		c.aoiOf[m.base+i], c.mgrOf[m.base+i], c.lastKind[m.base+i], c.lastKeep[m.base+i] = nil, nil, 0, 0
	}
	m.free, m.c = nil, nil
}

// submitPending hands the buffered calls to the library in call order: the
// entities' ids at their new slots first, then the ops, their Y and yaw
// filled in from the entities (SyncInfoSource) where the call had none.
func (c *Context) submitPending() {
	c.applyIDs()
	if len(c.ops) == 0 {
		return
	}
	for _, i := range c.resolve {
		a := c.aoiOf[c.ops[i].slot]
		src, ok := a.Data.(SyncInfoSource)
		if !ok {
			gwlog.Panicf("gpuaoi: %T has no AOISyncInfo() (INTEGRATION.md edit 2): the records need its Y and yaw", a.Data)
		}
		si := src.AOISyncInfo()
		c.ops[i].y, c.ops[i].yaw = C.float(si.Y), C.float(si.Yaw)
	}
	c.check(C.gw_submit(c.ctx, &c.ops[0], C.uint32_t(len(c.ops))))
	c.ops = c.ops[:0]
	c.resolve = c.resolve[:0]
	c.submitted = true
}

// Flush is called once per game tick for the whole process (edit 3): one
// submit, one tick, the canonical events of every space, then slot reclaim.
func (c *Context) Flush() {
	c.submitPending()
	var out C.gw_tick_out
	c.check(C.gw_tick(c.ctx, C.GW_TICK_COPY_TO_HOST, &out))
	c.submitted = false
	c.replay(&out)
	// a slot whose last op this tick was Leave is free again (its leave events
	// are delivered), or after the next Collect if the entity kept sync bits
	var gone []C.uint32_t
	for _, s := range c.touched {
		if c.lastKind[s] == C.GW_OP_LEAVE {
			m, a := c.mgrOf[s], c.aoiOf[s]
			if c.lastKeep[s] != 0 {
				m.parked[a] = true
				c.parked = append(c.parked, parkRef{m, a})
			} else {
				m.release(s, a)
				if c.ent[a] == nil { // destroyed (ClearIDs): its ids go with the slot
					gone = append(gone, C.uint32_t(s))
				}
			}
		}
		c.lastKind[s], c.lastKeep[s] = 0, 0
	}
	c.touched = c.touched[:0]
	if len(gone) > 0 {
		c.check(C.gw_clear_entity_ids(c.ctx, &gone[0], C.uint32_t(len(gone))))
	}
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

func (c *Context) info(a *aoi.AOI) *entInfo {
	e := c.ent[a]
	if e == nil {
		e = &entInfo{}
		c.ent[a] = e
	}
	return e
}

// SetEntityID registers an entity's EntityID (entity creation, where
// Entity.init calls aoi.InitAOI, Entity.go:210); the library maps it to the
// entity's slot while it is in an AOI space (client-record decode, records).
func (c *Context) SetEntityID(a *aoi.AOI, eid [16]byte) {
	c.info(a).eid = eid
	c.idDirty[a] = true
}

// SetClient attaches (gate > 0) or detaches (gate 0) the entity's client
// (GameClient{clientid, gateid}: Entity.SetClient / assignClient,
// GameClient.go:14-27).
func (c *Context) SetClient(a *aoi.AOI, clientid [16]byte, gate uint16) {
	e := c.info(a)
	e.cid, e.gate = clientid, gate
	c.idDirty[a] = true
}

// SetClientSyncing is Entity.SetClientSyncing (Entity.go:437-440): only
// entities that sync from their client take client position records
// (Entity.go:430-435).
func (c *Context) SetClientSyncing(a *aoi.AOI, on bool) {
	c.info(a).syncing = on
	c.idDirty[a] = true
}

// ClearIDs is entity destruction (Entity.destroyEntity, Entity.go:136-157),
// after its LeaveKeep(a, 0): its ids leave the library's tables when its slot
// is freed (gw_clear_entity_ids), so a late client record of it is dropped as
// EntityManager.go:451-455 drops one of a destroyed entity.
func (c *Context) ClearIDs(a *aoi.AOI) {
	delete(c.ent, a)
	delete(c.idDirty, a)
}

// applyIDs writes the registered ids, client and syncing flag of every entity
// that got a slot or changed them since the last call, at its slot, in one
// batch per table.
func (c *Context) applyIDs() {
	if len(c.idDirty) == 0 {
		return
	}
	var slots []C.uint32_t
	var eids, cids []byte
	var gates []C.uint16_t
	var on []C.uint8_t
	for a := range c.idDirty {
		m := c.cur[a]
		if m == nil {
			continue // not in an AOI space: the reference path handles it
		}
		s, ok := m.slotOf[a]
		if !ok || m.parked[a] {
			continue
		}
		e := c.ent[a]
		if e == nil {
			e = &entInfo{} // no id registered: zero ids, no client
		}
		slots = append(slots, C.uint32_t(s))
		eids = append(eids, e.eid[:]...)
		cids = append(cids, e.cid[:]...)
		gates = append(gates, C.uint16_t(e.gate))
		var b C.uint8_t
		if e.syncing {
			b = 1
		}
		on = append(on, b)
	}
	for a := range c.idDirty {
		delete(c.idDirty, a)
	}
	if len(slots) == 0 {
		return
	}
	n := C.uint32_t(len(slots))
	c.check(C.gw_set_entity_ids(c.ctx, &slots[0], unsafe.Pointer(&eids[0]), n))
	c.check(C.gw_set_client_ids(c.ctx, &slots[0], unsafe.Pointer(&cids[0]), n))
	c.check(C.gw_set_clients(c.ctx, &slots[0], &gates[0], n))
	c.check(C.gw_set_client_syncing(c.ctx, &slots[0], &on[0], n))
}

// ClientSync is HandleSyncPositionYawFromClient (GameService.go:395-407): the
// packet's payload after the msgtype, n records of eid[16] x y z yaw, decoded
// into Moved ops on the device side, after the calls buffered before it (call
// order).  Records of entities in AOI spaces of this context are applied
// here; the caller's reference loop handles the others (entities whose Space
// has no gpuaoi manager) and still sets e.Position / e.yaw of every record's
// entity for game code; toCaller counts the records of entities that left
// this context's spaces since their slot was last used.
func (c *Context) ClientSync(payload []byte) (toCaller uint32) {
	n := C.uint32_t(len(payload) / 32)
	if n == 0 {
		return 0
	}
	c.submitPending()
	var applied, left C.uint32_t
	c.check(C.gw_submit_client_sync(c.ctx, unsafe.Pointer(&payload[0]), n, &applied, &left))
	if applied > 0 {
		c.submitted = true
	}
	return uint32(left)
}

// Collect is CollectEntitySyncInfos (Entity.go:1221-1267): the records of
// every flagged entity, encoded as one packet per gate on the device
// (dispatchercluster.SelectByGateID(gate).SendPacket(pkt) in the reference).
// pkt is a slice of the library's pinned host buffer, valid until the next
// Collect: send copies what it keeps (netutil.Packet.AppendBytes does), no
// per-packet copy is made here.  Then the slots of entities that left with
// pending bits are freed.
func (c *Context) Collect(send func(gate uint16, pkt []byte)) {
	c.applyIDs()
	var so C.gw_sync_out
	c.check(C.gw_sync_collect(c.ctx, 0, &so))
	var wo C.gw_wire_out
	c.check(C.gw_sync_encode_wire(c.ctx, C.GW_WIRE_COPY_TO_HOST, &wo))
	if wo.n_packets > 0 {
		bytes := unsafe.Slice((*byte)(unsafe.Pointer(wo.bytes)), int(wo.n_bytes))
		gates := unsafe.Slice(wo.gate, int(wo.n_packets))
		offs := unsafe.Slice(wo.off, int(wo.n_packets)+1)
		for k, g := range gates {
			lo, hi := offs[k], offs[k+1]
			send(uint16(g), bytes[lo:hi:hi])
		}
	}
	c.unpark()
}

// unpark frees the slots of entities that left with pending sync bits and
// did not come back before this collect (their ids leave the tables with them).
func (c *Context) unpark() {
	var freed []C.uint32_t
	for _, p := range c.parked {
		if p.m.c == nil || !p.m.parked[p.a] {
			continue // re-entered, or freed already (space destroyed, a second park)
		}
		s := p.m.slotOf[p.a]
		p.m.release(s, p.a)
		freed = append(freed, C.uint32_t(s))
	}
	c.parked = c.parked[:0]
	if len(freed) > 0 {
		c.check(C.gw_clear_entity_ids(c.ctx, &freed[0], C.uint32_t(len(freed))))
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
