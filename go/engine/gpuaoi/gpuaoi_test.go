package gpuaoi

// Replays committed golden fixtures through the shim the way engine/entity
// drives it (INTEGRATION.md edits 1-5): ids and clients registered per entity,
// the initial population restored in bulk (Manager.Restore) or entered one by
// one, then per tick the server-side calls (Manager.Enter / MovedFlags /
// LeaveKeep / Sync, Y and yaw taken from the entity through AOISyncInfo) and
// the client position records (Context.ClientSync, 32-B records) in call
// order, Context.Flush (the OnEnterAOI / OnLeaveAOI callbacks) and
// Context.Collect (the game->gate packets).  Compared with the fixture: every
// tick's callbacks (canonical net events), the number of records and the
// SHA-256 of the packets after putting each packet's records in canonical
// order (the reference emits an entity's neighbour records in Go map order,
// so only that order is free).  server_y_s13 has a non-zero Y and yaw in every
// position, so each record's payload is checked against the fixture's.
// The fixtures come from the repository's oracle (tests/golden/*.npz); `go
// generate` exports them into testdata/.  Needs the MI355X: gw_init fails
// loudly without a HIP device.

//go:generate python3 ../../third_party/goworld_amd/tests/golden/export_gwh.py testdata cfg1_walk adversarial_s11 dyadic_hot_2k server_y_s13

import (
	"bytes"
	"crypto/sha256"
	"encoding/binary"
	"math"
	"os"
	"path/filepath"
	"sort"
	"testing"

	"github.com/xiaonanln/go-aoi"
	"github.com/xiaonanln/goworld/engine/proto"
)

type gwhOp struct {
	kind, flags  uint8
	slot         uint32
	x, y, z, yaw float32
}

type gwhTrace struct {
	capacity uint32
	d        float32
	bounds   [4]float32
	init     []gwhOp // slot, x, y, z, yaw of the initial population
	gates    []uint16
	ticks    [][]gwhOp
}

func readTrace(path string) (*gwhTrace, error) {
	raw, err := os.ReadFile(path)
	if err != nil {
		return nil, err
	}
	r := bytes.NewReader(raw)
	le := binary.LittleEndian
	var hdr struct {
		Magic    [4]byte
		Capacity uint32
		D        float32
		Bounds   [4]float32
		NInit    uint32
		NTicks   uint32
	}
	if err := binary.Read(r, le, &hdr); err != nil {
		return nil, err
	}
	tr := &gwhTrace{capacity: hdr.Capacity, d: hdr.D, bounds: hdr.Bounds}
	for i := uint32(0); i < hdr.NInit; i++ {
		var e struct {
			Slot         uint32
			X, Y, Z, Yaw float32
		}
		if err := binary.Read(r, le, &e); err != nil {
			return nil, err
		}
		tr.init = append(tr.init, gwhOp{slot: e.Slot, x: e.X, y: e.Y, z: e.Z, yaw: e.Yaw})
	}
	tr.gates = make([]uint16, hdr.Capacity)
	if err := binary.Read(r, le, tr.gates); err != nil {
		return nil, err
	}
	for t := uint32(0); t < hdr.NTicks; t++ {
		var n uint32
		if err := binary.Read(r, le, &n); err != nil {
			return nil, err
		}
		ops := make([]gwhOp, n)
		for i := range ops {
			var o struct {
				Kind, Flags  uint8
				Reserved     uint16
				Slot         uint32
				X, Y, Z, Yaw float32
			}
			if err := binary.Read(r, le, &o); err != nil {
				return nil, err
			}
			ops[i] = gwhOp{kind: o.Kind, flags: o.Flags, slot: o.Slot, x: o.X, y: o.Y, z: o.Z, yaw: o.Yaw}
		}
		tr.ticks = append(tr.ticks, ops)
	}
	return tr, nil
}

type event struct{ watcher, target uint32 }

func readEvents(path string, ticks int) ([][2][]event, error) {
	raw, err := os.ReadFile(path)
	if err != nil {
		return nil, err
	}
	r := bytes.NewReader(raw)
	out := make([][2][]event, ticks)
	for t := 0; t < ticks; t++ {
		for k := 0; k < 2; k++ {
			var n uint64
			if err := binary.Read(r, binary.LittleEndian, &n); err != nil {
				return nil, err
			}
			w := make([]uint32, 2*n) // (watcher, target) pairs; binary.Read cannot set unexported fields
			if err := binary.Read(r, binary.LittleEndian, w); err != nil {
				return nil, err
			}
			ev := make([]event, n)
			for i := range ev {
				ev[i] = event{w[2*i], w[2*i+1]}
			}
			out[t][k] = ev
		}
	}
	return out, nil
}

type wireWant struct {
	nRec uint64
	sha  [32]byte
}

func readWire(path string, ticks int) ([]wireWant, error) {
	raw, err := os.ReadFile(path)
	if err != nil {
		return nil, err
	}
	r := bytes.NewReader(raw)
	out := make([]wireWant, ticks)
	for t := range out {
		if err := binary.Read(r, binary.LittleEndian, &out[t].nRec); err != nil {
			return nil, err
		}
		if _, err := r.Read(out[t].sha[:]); err != nil {
			return nil, err
		}
	}
	return out, nil
}

// fixedUUID is GenFixedUUID (engine/uuid/uuid.go:48-59): the base64 (A-Z a-z
// 0-9 _ .) of 12 bytes holding v big-endian in the last four.
func fixedUUID(v uint32) (out [16]byte) {
	const alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_."
	var b [12]byte
	binary.BigEndian.PutUint32(b[8:], v)
	for i, o := 0, 0; i < 12; i, o = i+3, o+4 {
		out[o] = alpha[b[i]>>2]
		out[o+1] = alpha[(b[i]&3)<<4|b[i+1]>>4]
		out[o+2] = alpha[(b[i+1]&15)<<2|b[i+2]>>6]
		out[o+3] = alpha[b[i+2]&63]
	}
	return
}

// testEntity stands in for *entity.Entity: its id is the trace slot; pos is
// e.Position / e.yaw (AOISyncInfo, INTEGRATION.md edit 2).
type testEntity struct {
	id  uint32
	a   aoi.AOI
	pos proto.EntitySyncInfo
	log *[2][]event
}

func (e *testEntity) OnEnterAOI(o *aoi.AOI) {
	e.log[0] = append(e.log[0], event{e.id, o.Data.(*testEntity).id})
}
func (e *testEntity) OnLeaveAOI(o *aoi.AOI) {
	e.log[1] = append(e.log[1], event{e.id, o.Data.(*testEntity).id})
}
func (e *testEntity) AOISyncInfo() proto.EntitySyncInfo { return e.pos }

func canonical(ev []event) []event {
	sort.Slice(ev, func(i, j int) bool {
		if ev[i].watcher != ev[j].watcher {
			return ev[i].watcher < ev[j].watcher
		}
		return ev[i].target < ev[j].target
	})
	return ev
}

func equalEvents(a, b []event) bool {
	if len(a) != len(b) {
		return false
	}
	for i := range a {
		if a[i] != b[i] {
			return false
		}
	}
	return true
}

type wireRec struct {
	gate            uint16
	watcher, entity uint32
	raw             []byte // the 48-B record
}

// canonicalWire parses the tick's packets (u16 1502, u16 gate, 48-B records
// clientid(watcher) eid(entity) x y z yaw) and re-encodes them with the
// records in (gate(watcher), entity, watcher) order, as the fixture's
// wire_sha was taken.
func canonicalWire(t *testing.T, pkts map[uint16][]byte, eid, cid map[[16]byte]uint32) ([]byte, uint64) {
	var recs []wireRec
	for gate, p := range pkts {
		if len(p) < 4 || binary.LittleEndian.Uint16(p) != 1502 || binary.LittleEndian.Uint16(p[2:]) != gate ||
			(len(p)-4)%48 != 0 {
			t.Fatalf("gate %d: bad packet header or length %d", gate, len(p))
		}
		for q := 4; q < len(p); q += 48 {
			var c, e [16]byte
			copy(c[:], p[q:q+16])
			copy(e[:], p[q+16:q+32])
			w, ok1 := cid[c]
			en, ok2 := eid[e]
			if !ok1 || !ok2 {
				t.Fatalf("gate %d: record with an unknown client or entity id", gate)
			}
			recs = append(recs, wireRec{gate, w, en, p[q : q+48]})
		}
	}
	sort.Slice(recs, func(i, j int) bool {
		a, b := recs[i], recs[j]
		if a.gate != b.gate {
			return a.gate < b.gate
		}
		if a.entity != b.entity {
			return a.entity < b.entity
		}
		return a.watcher < b.watcher
	})
	var out []byte
	for i := 0; i < len(recs); {
		j := i
		for j < len(recs) && recs[j].gate == recs[i].gate {
			j++
		}
		out = binary.LittleEndian.AppendUint16(out, 1502)
		out = binary.LittleEndian.AppendUint16(out, recs[i].gate)
		for _, r := range recs[i:j] {
			out = append(out, r.raw...)
		}
		i = j
	}
	return out, uint64(len(recs))
}

func TestReplayGolden(t *testing.T) {
	for _, tc := range []struct {
		name    string
		restore bool
	}{{"cfg1_walk", true}, {"adversarial_s11", false}, {"dyadic_hot_2k", true}, {"server_y_s13", true},
		{"server_y_s13", false}} {
		tc := tc
		t.Run(tc.name, func(t *testing.T) { replayGolden(t, tc.name, tc.restore) })
	}
}

func replayGolden(t *testing.T, name string, restore bool) {
	tr, err := readTrace(filepath.Join("testdata", name+".gwh"))
	if os.IsNotExist(err) {
		t.Skip("run `go generate` first (exports the fixtures into testdata/)")
	}
	if err != nil {
		t.Fatal(err)
	}
	want, err := readEvents(filepath.Join("testdata", name+".events"), len(tr.ticks))
	if err != nil {
		t.Fatal(err)
	}
	wire, err := readWire(filepath.Join("testdata", name+".wire"), len(tr.ticks))
	if err != nil {
		t.Fatal(err)
	}
	c := NewContext(0)
	defer c.Close()
	// a first size below the trace's: the manager grows (and may move) the space
	m := c.NewManager(aoi.Coord(tr.d), tr.capacity/4+1, tr.bounds[0], tr.bounds[1], tr.bounds[2], tr.bounds[3])
	var log [2][]event
	ents := make([]*testEntity, tr.capacity)
	eid, cid := map[[16]byte]uint32{}, map[[16]byte]uint32{}
	for i := range ents {
		e := &testEntity{id: uint32(i), log: &log}
		ents[i] = e
		aoi.InitAOI(&e.a, aoi.Coord(tr.d), e, e)
		// entity creation and client attach (Entity.go:210, GameClient.go:14-27, Entity.go:437-440)
		ei, ci := fixedUUID(uint32(i)), fixedUUID(uint32(i)|0x80000000)
		eid[ei], cid[ci] = uint32(i), uint32(i)
		c.SetEntityID(&e.a, ei)
		if tr.gates[i] != 0 {
			c.SetClient(&e.a, ci, tr.gates[i])
		}
		c.SetClientSyncing(&e.a, true)
	}
	if restore { // the restore path (Space.go:209-214) in one call
		rs := make([]RestoreEntry, len(tr.init))
		for k, p := range tr.init {
			ents[p.slot].pos = proto.EntitySyncInfo{X: p.x, Y: p.y, Z: p.z, Yaw: p.yaw}
			rs[k] = RestoreEntry{A: &ents[p.slot].a, X: p.x, Y: p.y, Z: p.z, Yaw: p.yaw}
		}
		m.Restore(rs)
	} else { // N Enter calls and a flush
		for _, p := range tr.init {
			ents[p.slot].pos = proto.EntitySyncInfo{X: p.x, Y: p.y, Z: p.z, Yaw: p.yaw}
			m.Enter(&ents[p.slot].a, aoi.Coord(p.x), aoi.Coord(p.z))
		}
		c.Flush()
	}
	// the load's callbacks: every pair both ways, exactly the final relation
	got := canonical(append([]event(nil), log[0]...))
	for k := 1; k < len(got); k++ {
		if got[k] == got[k-1] {
			t.Fatalf("%s: load fired %v twice", name, got[k])
		}
	}
	log[0], log[1] = log[0][:0], log[1][:0]
	var payload []byte // consecutive client records (MT_SYNC_POSITION_YAW_FROM_CLIENT)
	sendClient := func() {
		if len(payload) > 0 {
			if left := c.ClientSync(payload); left != 0 {
				t.Fatalf("%s: %d client records left to the caller", name, left)
			}
			payload = payload[:0]
		}
	}
	for k, ops := range tr.ticks {
		for _, o := range ops {
			e := ents[o.slot]
			a := &e.a
			if o.kind == 2 && o.flags == SifNeighborClients { // a client's move (fromClient = true)
				e.pos = proto.EntitySyncInfo{X: o.x, Y: o.y, Z: o.z, Yaw: o.yaw}
				var rec [32]byte
				id := fixedUUID(o.slot)
				copy(rec[:16], id[:])
				binary.LittleEndian.PutUint32(rec[16:], math.Float32bits(o.x))
				binary.LittleEndian.PutUint32(rec[20:], math.Float32bits(o.y))
				binary.LittleEndian.PutUint32(rec[24:], math.Float32bits(o.z))
				binary.LittleEndian.PutUint32(rec[28:], math.Float32bits(o.yaw))
				payload = append(payload, rec[:]...)
				continue
			}
			sendClient()
			switch o.kind {
			case 1:
				e.pos = proto.EntitySyncInfo{X: o.x, Y: o.y, Z: o.z, Yaw: o.yaw}
				m.Enter(a, aoi.Coord(o.x), aoi.Coord(o.z))
			case 2:
				// setPositionYaw: Space.move (the manager call), then e.yaw (Entity.go:1189-1205)
				e.pos.X, e.pos.Y, e.pos.Z = o.x, o.y, o.z
				m.MovedFlags(a, aoi.Coord(o.x), aoi.Coord(o.z), o.flags)
				e.pos.Yaw = o.yaw
			case 3:
				m.LeaveKeep(a, o.flags)
			case 4:
				e.pos.Yaw = o.yaw
				m.Sync(a, o.x, o.y, o.z, o.yaw, o.flags)
			}
		}
		sendClient()
		c.Flush()
		for j, kind := range []string{"enter", "leave"} {
			got := canonical(append([]event(nil), log[j]...))
			if !equalEvents(got, want[k][j]) {
				t.Fatalf("%s tick %d: %s events differ (%d vs %d)", name, k, kind, len(got), len(want[k][j]))
			}
		}
		log[0], log[1] = log[0][:0], log[1][:0]
		pkts := map[uint16][]byte{}
		c.Collect(func(gate uint16, pkt []byte) {
			if _, dup := pkts[gate]; dup {
				t.Fatalf("%s tick %d: two packets for gate %d", name, k, gate)
			}
			pkts[gate] = append([]byte(nil), pkt...) // valid until the next Collect
		})
		b, n := canonicalWire(t, pkts, eid, cid)
		if n != wire[k].nRec {
			t.Fatalf("%s tick %d: %d records, want %d", name, k, n, wire[k].nRec)
		}
		if sha256.Sum256(b) != wire[k].sha {
			t.Fatalf("%s tick %d: game->gate packets differ from the fixture", name, k)
		}
	}
}
