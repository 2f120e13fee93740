"""GPU: the HIP path (through the C ABI) against the committed golden fixtures.

Small fixtures (tests/golden/*.npz: config #1 walks, rounding-edge churn
traces, a dyadic hotspot trace with 3 gates and client-less entities): every
tick's canonical enter / leave events byte for byte, the sync records of every
collect (count + SHA-256 of the canonical bytes, tick 0 in full) and the final
InterestedIn sets.  Large configs (#2 100k, #3 1M, #4 10k spaces x 1k in one context;
tests/golden/digests.json): per tick event and record digests, on traces
regenerated from their seeds (input hash checked first).  No oracle runs here: the expected outputs are
data.
"""
import numpy as np
import pytest

import golden_data as G
from goworld_amd import gpuaoi
from goworld_amd import traces as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    g = []

    def make():
        c = gpuaoi.GpuAOI(0)
        g.append(c)
        return c
    yield make
    for c in g:
        c.close()


def canonical(recs: np.ndarray, gates: np.ndarray) -> np.ndarray:
    """Records in the fixtures' (gate(watcher), entity, watcher) order via one
    u64 key (gate 16 | entity 24 | watcher 24 bits).  The GPU stream is already
    in (gate, entity) order (checked) with only the watchers of an entity in
    grid order (test_gpu_parity checks that order exactly), so the stable
    (run-merging) sort is near linear even for the 1M config's load collect
    (~1.5e8 records)."""
    if len(recs) == 0:
        return recs
    assert len(gates) <= 1 << 24
    ge = (gates[recs["watcher"]].astype(np.uint64) << np.uint64(24)) | recs["entity"].astype(np.uint64)
    assert np.all(ge[1:] >= ge[:-1]), "record stream not grouped by (gate, entity)"
    key = (ge << np.uint64(24)) | recs["watcher"].astype(np.uint64)
    return recs[np.argsort(key, kind="stable")]


@pytest.mark.parametrize("name", G.SMALL)
def test_small_fixture(gpu, name):
    fx = G.Fixture(name)
    tr = fx.trace
    g = gpu()
    sid, base = gpuaoi.load_space(g, tr)
    assert base == 0
    for t, ops in enumerate(tr.ticks):
        g.submit(ops)
        res = g.tick()
        ee, ll = fx.events(t)
        assert res.enter.tobytes() == ee.tobytes(), f"{name} tick {t}: enter events"
        assert res.leave.tobytes() == ll.tobytes(), f"{name} tick {t}: leave events"
        r = g.sync_collect()
        got = canonical(r.records, tr.gates)
        assert r.n_rec == fx.n_rec(t), f"{name} tick {t}: record count"
        assert G.sha(got) == fx.rec_sha(t), f"{name} tick {t}: records"
        if t == 0:
            assert got.tobytes() == fx.rec0.tobytes()
    assert g.total_neighbors() == fx.nbr_total
    assert G.neighbour_sha(g.neighbors(s) for s in range(tr.capacity)) == fx.nbr_sha
    g.close()


@pytest.mark.parametrize("name", list(G.DIGEST_TRACES))
def test_large_config_digests(gpu, name):
    d = G.digests()[name]
    tr = G.DIGEST_TRACES[name]()
    assert G.trace_input_sha(tr) == d["input_sha"], "trace generator changed (not a parity failure)"
    g = gpu()
    gpuaoi.load_space(g, tr)
    for t, ops in enumerate(tr.ticks):
        exp = d["ticks"][t]
        g.submit(ops)
        res = g.tick()
        assert (res.n_enter, res.n_leave) == (exp["n_enter"], exp["n_leave"])
        assert G.sha(res.enter) == exp["enter_sha"] and G.sha(res.leave) == exp["leave_sha"]
        r = g.sync_collect()
        assert r.n_rec == exp["n_rec"]
        recs = canonical(r.records, tr.gates)
        del r
        assert G.sha(recs) == exp["rec_sha"], f"{name} tick {t}: records"
        del recs
    if "nbr_total" in d:
        assert g.total_neighbors() == d["nbr_total"]
    g.close()


@pytest.mark.parametrize("name", list(G.MULTI_DIGEST_TRACES))
def test_many_spaces_config4_digests(gpu, name):
    """Config #4 at its workload: 10k spaces x 1k entities in one context, every
    tick one gw_tick over all of them; per tick the digests of the whole
    context's canonical events and records (tests/golden/digests.json, from
    per-space ORC_SEQRULE + gridmt runs merged in global slot order)."""
    d = G.digests()[name]
    trs = G.MULTI_DIGEST_TRACES[name]()
    assert G.multi_input_sha(trs) == d["input_sha"], "trace generator changed (not a parity failure)"
    assert len(trs) == d["spaces"]
    g = gpu()
    bases = []
    for tr in trs:
        _, base = gpuaoi.load_space(g, tr)
        bases.append(base)
    assert bases == list(np.cumsum([0] + [tr.capacity for tr in trs[:-1]]))
    gates = np.concatenate([tr.gates for tr in trs])
    g.sync_collect()                                  # the load's collect (not digested)
    for t in range(len(trs[0].ticks)):
        exp = d["ticks"][t]
        ops = np.concatenate([T.with_global_slots(tr.ticks[t], b) for tr, b in zip(trs, bases)])
        g.submit(ops)
        res = g.tick()
        assert (res.n_enter, res.n_leave) == (exp["n_enter"], exp["n_leave"])
        assert G.sha(res.enter) == exp["enter_sha"] and G.sha(res.leave) == exp["leave_sha"]
        r = g.sync_collect()
        assert r.n_rec == exp["n_rec"]
        recs = canonical(r.records, gates)
        del r
        assert G.sha(recs) == exp["rec_sha"], f"{name} tick {t}: records"
        del recs
    assert g.total_neighbors() == d["nbr_total"]
    g.close()


@pytest.mark.parametrize("cap", [1, 3])
def test_grid_stride_passes_capped(gpu, cap, monkeypatch):
    """The flatten and bucket tile passes loop grid-stride when a tick has more
    items than their grid (sized by the last tick's items).  GW_GRID_CAP caps
    those grids to `cap` blocks, so every block runs many chunk / tile
    iterations (reusing its LDS histograms and staging): the config #2 digests
    (100k entities, ~10^5 items per tick = dozens of 8192-item tiles) must
    still match."""
    monkeypatch.setenv("GW_GRID_CAP", str(cap))
    name = "config2_100k"
    d = G.digests()[name]
    tr = G.DIGEST_TRACES[name]()
    g = gpu()                                   # gw_init reads GW_GRID_CAP
    monkeypatch.delenv("GW_GRID_CAP")
    gpuaoi.load_space(g, tr)
    for t, ops in enumerate(tr.ticks):
        exp = d["ticks"][t]
        g.submit(ops)
        res = g.tick()
        assert (res.n_enter, res.n_leave) == (exp["n_enter"], exp["n_leave"])
        assert G.sha(res.enter) == exp["enter_sha"] and G.sha(res.leave) == exp["leave_sha"], f"tick {t}"
        assert res.n_enter + res.n_leave > 2 * 8192                # many chunks per wave, >= 2 tiles
        r = g.sync_collect()
        assert G.sha(canonical(r.records, tr.gates)) == exp["rec_sha"], f"tick {t}: records"
    g.close()


@pytest.mark.parametrize("pair_max", [96, 1 << 20])
def test_mover_pairing_modes(gpu, pair_max, monkeypatch):
    """With GW_PAIR_MAX > 0 the diff runs two short-list movers per wave
    (k_mover_pair; off by default since it measured slower at config #3) and
    longer ones one per wave (mover_one): the mixed path (96) and pairing every
    mover give the same config #2 digests as the default one-wave path."""
    monkeypatch.setenv("GW_PAIR_MAX", str(pair_max))
    name = "config2_100k"
    d = G.digests()[name]
    tr = G.DIGEST_TRACES[name]()
    g = gpu()                                   # gw_init reads GW_PAIR_MAX
    monkeypatch.delenv("GW_PAIR_MAX")
    gpuaoi.load_space(g, tr)
    for t, ops in enumerate(tr.ticks):
        exp = d["ticks"][t]
        g.submit(ops)
        res = g.tick()
        assert (res.n_enter, res.n_leave) == (exp["n_enter"], exp["n_leave"])
        assert G.sha(res.enter) == exp["enter_sha"] and G.sha(res.leave) == exp["leave_sha"], f"tick {t}"
        r = g.sync_collect()
        assert G.sha(canonical(r.records, tr.gates)) == exp["rec_sha"], f"tick {t}: records"
    g.close()


def test_pair_mode_fallback_digests(gpu, monkeypatch):
    """The paired diff (k_mover_pair, GW_PAIR_MAX) with GW_HALF_ROWS=0: every
    pair falls back to one mover_one walk per entry; config #2 digests."""
    monkeypatch.setenv("GW_PAIR_MAX", "96")
    monkeypatch.setenv("GW_HALF_ROWS", "0")
    name = "config2_100k"
    d = G.digests()[name]
    tr = G.DIGEST_TRACES[name]()
    g = gpu()
    monkeypatch.delenv("GW_PAIR_MAX")
    monkeypatch.delenv("GW_HALF_ROWS")
    gpuaoi.load_space(g, tr)
    for t, ops in enumerate(tr.ticks):
        exp = d["ticks"][t]
        g.submit(ops)
        res = g.tick()
        assert G.sha(res.enter) == exp["enter_sha"] and G.sha(res.leave) == exp["leave_sha"], f"tick {t}"
        r = g.sync_collect()
        assert G.sha(canonical(r.records, tr.gates)) == exp["rec_sha"], f"tick {t}: records"
    g.close()
