"""Export golden fixtures for the Go shim's replay test
(go/engine/gpuaoi/gpuaoi_test.go, run by `go generate` there).

usage: python3 tests/golden/export_gwh.py OUTDIR NAME...
  OUTDIR/NAME.gwh     the trace in the c_harness input format (tests/c_harness.c)
  OUTDIR/NAME.events  per tick: u64 n_enter, enters (u32 watcher, u32 target),
                      u64 n_leave, leaves -- the fixture's canonical net events
  OUTDIR/NAME.wire    per tick: u64 records of the collect, the 32-byte SHA-256
                      of the game->gate packets with the records in canonical
                      (gate(watcher), entity, watcher) order
Data only: the expected outputs are the committed fixtures' (tests/golden/*.npz).
"""
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))              # tests/
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))   # repo root

import golden_data as G                                 # noqa: E402
from test_c_harness import _write_input                 # noqa: E402


def main(argv):
    out, names = argv[0], argv[1:]
    os.makedirs(out, exist_ok=True)
    for name in names:
        fx = G.Fixture(name)
        _write_input(os.path.join(out, f"{name}.gwh"), fx)
        with open(os.path.join(out, f"{name}.events"), "wb") as f:
            for t in range(fx.ticks):
                e, l = fx.events(t)
                for a in (e, l):
                    f.write(struct.pack("<Q", len(a)))
                    f.write(a.tobytes())
        with open(os.path.join(out, f"{name}.wire"), "wb") as f:
            for t in range(fx.ticks):
                f.write(struct.pack("<Q", fx.n_rec(t)))
                f.write(bytes.fromhex(fx.wire_sha(t)))


if __name__ == "__main__":
    main(sys.argv[1:])
