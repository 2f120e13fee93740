package gpuaoi

// Replays committed golden fixtures through the shim (Manager.Enter / Moved /
// Leave / Sync buffered, Context.Flush, the OnEnterAOI / OnLeaveAOI callbacks)
// and compares every tick's callbacks with the fixture's canonical net events.
// The fixtures come from the repository's oracle (tests/golden/*.npz); `go
// generate` exports them (trace + expected events) into testdata/.  Needs the
// MI355X: gw_init fails loudly without a HIP device.

//go:generate python3 ../../third_party/goworld_amd/tests/golden/export_gwh.py testdata cfg1_walk adversarial_s11 dyadic_hot_2k

import (
	"bytes"
	"encoding/binary"
	"os"
	"path/filepath"
	"sort"
	"testing"

	"github.com/xiaonanln/go-aoi"
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

// testEntity stands in for *entity.Entity: its id is the trace slot.
type testEntity struct {
	id  uint32
	a   aoi.AOI
	log *[2][]event
}

func (e *testEntity) OnEnterAOI(o *aoi.AOI) {
	e.log[0] = append(e.log[0], event{e.id, o.Data.(*testEntity).id})
}
func (e *testEntity) OnLeaveAOI(o *aoi.AOI) {
	e.log[1] = append(e.log[1], event{e.id, o.Data.(*testEntity).id})
}

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

func TestReplayGolden(t *testing.T) {
	for _, name := range []string{"cfg1_walk", "adversarial_s11", "dyadic_hot_2k"} {
		t.Run(name, func(t *testing.T) { replayGolden(t, name) })
	}
}

func replayGolden(t *testing.T, name string) {
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
	c := NewContext(0)
	defer c.Close()
	// a first size below the trace's: the manager grows (and may move) the space
	m := c.NewManager(aoi.Coord(tr.d), tr.capacity/4+1, tr.bounds[0], tr.bounds[1], tr.bounds[2], tr.bounds[3])
	var log [2][]event
	ents := make([]*testEntity, tr.capacity)
	for i := range ents {
		ents[i] = &testEntity{id: uint32(i), log: &log}
		aoi.InitAOI(&ents[i].a, aoi.Coord(tr.d), ents[i], ents[i])
	}
	for _, p := range tr.init { // the restore path: N Enter calls (Space.go:209-214)
		m.Enter(&ents[p.slot].a, aoi.Coord(p.x), aoi.Coord(p.z))
	}
	c.Flush()
	for i, e := range ents { // clients after the load, by the manager's slot of each entity
		if tr.gates[i] != 0 {
			if s, ok := m.Slot(&e.a); ok {
				c.SetClient(s, tr.gates[i])
			}
		}
	}
	log[0], log[1] = log[0][:0], log[1][:0]
	for k, ops := range tr.ticks {
		for _, o := range ops {
			a := &ents[o.slot].a
			switch o.kind {
			case 1:
				m.Enter(a, aoi.Coord(o.x), aoi.Coord(o.z))
			case 2:
				m.MovedFlags(a, aoi.Coord(o.x), aoi.Coord(o.z), o.flags)
			case 3:
				m.LeaveKeep(a, o.flags)
			case 4:
				m.Sync(a, o.x, o.y, o.z, o.yaw, o.flags)
			}
		}
		c.Flush()
		for j, kind := range []string{"enter", "leave"} {
			got := canonical(append([]event(nil), log[j]...))
			if !equalEvents(got, want[k][j]) {
				t.Fatalf("%s tick %d: %s events differ (%d vs %d)", name, k, kind, len(got), len(want[k][j]))
			}
		}
		log[0], log[1] = log[0][:0], log[1][:0]
	}
}
