"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every
symbol include/gpuaoi.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np

from goworld_amd import gpuaoi, traces

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "gpuaoi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gw_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = gpuaoi.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), f"{s} declared in gpuaoi.h but not exported"
    assert set(syms) == set(gpuaoi.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", gpuaoi.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), s


def test_abi_version_and_layouts():
    assert gpuaoi.lib().gw_abi_version() == 15
    assert ctypes.sizeof(gpuaoi.CtxInfo) == 24
    assert ctypes.sizeof(gpuaoi.WireOut) == 7 * 8
    assert ctypes.sizeof(gpuaoi.Xfer) == 40 and ctypes.sizeof(gpuaoi.WorldGeom) == 24
    assert gpuaoi.FANOUT_DTYPE.itemsize == 12
    assert ctypes.sizeof(gpuaoi.MsgOut) == 7 * 8
    assert ctypes.sizeof(gpuaoi.HaloDst) == 24
    assert traces.LONG_DTYPE.itemsize == 48            # gw_long_move
    assert traces.OP_DTYPE.itemsize == 24
    assert gpuaoi.EVENT_DTYPE.itemsize == 8
    assert gpuaoi.REC_DTYPE.itemsize == 24
    assert ctypes.sizeof(gpuaoi.TickOut) == 4 * 8 + 7 * 8 + 8 * 2


def test_library_is_gfx950_code_object():
    blob = open(gpuaoi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob   # gfx950 only, no multi-arch dispatch


def test_init_without_gpu_fails_loudly():
    """No HIP device in this container: gw_init must fail, not fall back."""
    import torch
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    rc = gpuaoi.lib().gw_init(0, ctypes.byref(h))
    assert rc != 0 and not h.value


def test_trace_determinism():
    a = traces.config2(ticks=2, n=5000)
    b = traces.config2(ticks=2, n=5000)
    assert np.array_equal(a.init_x, b.init_x) and a.ticks[1].tobytes() == b.ticks[1].tobytes()
    # dyadic grid: x*128 integral, |x| < 2**17, so x +- d is exact in float32
    x = a.ticks[1]["x"].astype(np.float64)
    assert np.all(x * 128 == np.round(x * 128)) and np.all(np.abs(x) < 2 ** 17)
    # movers are distinct per tick
    assert len(np.unique(a.ticks[0]["slot"])) == len(a.ticks[0])
