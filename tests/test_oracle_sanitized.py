"""CPU: the oracle and the plain-C harness under AddressSanitizer +
UndefinedBehaviorSanitizer ("ASan/UBSan on the CPU restatement
and harness").

`make -C oracle san` builds oracle/orc.c with the sanitizers into a standalone
replay driver (oracle/orc_replay.c, no Python in the process), and `make san`
builds tests/c_harness.c likewise.  Every small golden fixture is replayed
through each oracle engine (XZList restatement, brute force, seq rule): any
out-of-bounds access, use after free, leak, signed overflow, misaligned or
invalid shift aborts the driver (-fno-sanitize-recover=all), and its outputs
must still equal the fixtures (events, records, wire bytes, neighbour lists)
and the unsanitized library's client-message and fan-out counts.  The
harness runs its no-device path (input parsing, gw_init failing loudly).
"""
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

import golden_data as G
from oracle import pyorc
from test_c_harness import _write_input

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "oracle", "build", "san", "orc_replay")
HARNESS_SAN = os.path.join(ROOT, "goworld_amd", "lib", "c_harness_san")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    assert os.path.exists(REPLAY)
    return REPLAY


def _read(path, ticks, cap):
    b = open(path, "rb").read()
    p = 0

    def take(n):
        nonlocal p
        v = b[p:p + n]
        p += n
        return v

    def u64():
        return struct.unpack("<Q", take(8))[0]
    out = []
    for _ in range(ticks):
        e = np.frombuffer(take(8 * u64()), G.EVENT_DTYPE)
        l = np.frombuffer(take(8 * u64()), G.EVENT_DTYPE)
        r = np.frombuffer(take(24 * u64()), G.REC_DTYPE)
        w = take(u64())
        out.append((e, l, r, w, u64(), u64(), u64()))
    total = u64()
    lists = []
    for _ in range(cap):
        k = struct.unpack("<I", take(4))[0]
        lists.append(np.frombuffer(take(4 * k), np.uint32))
    assert p == len(b)
    return out, total, lists


@pytest.mark.parametrize("mode", [pyorc.XZLIST, pyorc.BRUTE, pyorc.SEQRULE])
@pytest.mark.parametrize("name", G.SMALL)
def test_sanitized_oracle_reproduces_fixture(san_build, tmp_path, name, mode):
    fx = G.Fixture(name)
    tr = fx.trace
    _write_input(tmp_path / "in.bin", fx)
    r = subprocess.run([san_build, str(mode), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, env=SAN_ENV, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    out, total, lists = _read(tmp_path / "out.bin", fx.ticks, tr.capacity)
    # the unsanitized library on the same trace: client-message and fan-out counts
    o = pyorc.OracleSpace(tr.capacity, tr.d, mode)
    pyorc.load_trace(o, tr)
    for t, (e, l, rec, wire, ncr, nde, nfo) in enumerate(out):
        ee, ll = fx.events(t)
        assert e.tobytes() == ee.tobytes() and l.tobytes() == ll.tobytes(), f"{name} tick {t}: events"
        assert len(rec) == fx.n_rec(t) and G.sha(rec) == fx.rec_sha(t), f"{name} tick {t}: records"
        if t == 0:
            assert rec.tobytes() == fx.rec0.tobytes()
        assert hashlib.sha256(wire).hexdigest() == fx.wire_sha(t), f"{name} tick {t}: wire bytes"
        ops = tr.ticks[t]
        assert o.tick(ops) == 0
        cr, de = o.client_events()
        calls = np.array([s for s in ops["slot"] if o.present(int(s))], np.uint32)
        assert (ncr, nde, nfo) == (len(cr), len(de), len(o.fanout(calls))), f"{name} tick {t}: messages"
        o.collect()
    assert total == fx.nbr_total
    assert G.neighbour_sha(lists) == fx.nbr_sha


def test_sanitized_harness_fails_loudly_without_a_device(tmp_path):
    """The plain-C ABI caller built with ASan + UBSan: input parsing and the
    no-device error path run clean (the HIP runtime it loads is not ours, so
    leak checking is off for it)."""
    subprocess.run(["make", "-s", "-C", ROOT, "san"], check=True)
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present: the no-device path is not reachable")
    fx = G.Fixture("cfg1_walk")
    _write_input(tmp_path / "in.bin", fx)
    env = dict(SAN_ENV, ASAN_OPTIONS="halt_on_error=1:detect_leaks=0")
    r = subprocess.run([HARNESS_SAN, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 2 and "gw_init" in r.stderr, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr
    r = subprocess.run([HARNESS_SAN, str(tmp_path / "missing.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2 and "Sanitizer" not in r.stderr
