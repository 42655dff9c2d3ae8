"""Parity of the HIP path (librbhip.so through the C-ABI) against the goldens
produced by the reference's own functions and against the oracle.

Bar: fp64 bit-exact (contacts AND state) — the kernels keep the reference's
operation order; fp32 bit-exact against the fp32 restatement; fp32 vs fp64
within the SURVEY §8d sweep tolerance."""
import ctypes as C
import time

import numpy as np
import pytest

from conftest import NBODY_GOLDENS, golden_scene, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


# ---------------------------------------------------------------- KATs
def test_kat_impulse_device_bit_exact(rb):
    g = load_golden("kat_impulse")
    out = rb.kat_impulse(g["inp"])
    bad = np.nonzero((out != g["out"]).any(1))[0]
    assert bad.size == 0, f"{bad.size} KAT rows differ, first {bad[:5]}: {out[bad[:1]]} vs {g['out'][bad[:1]]}"


def test_kat_inertia_device_bit_exact(rb):
    g = load_golden("kat_inertia")
    out = rb.kat_inertia(g["inp"])
    assert np.array_equal(out, g["out"])


def test_kat_f32_matches_f32_restatement(rb, oracle):
    g = load_golden("kat_impulse")
    assert np.array_equal(rb.kat_impulse(g["inp"], dtype="f32"), oracle.kat_impulse(g["inp"], dtype="f32"))
    g = load_golden("kat_inertia")
    assert np.array_equal(rb.kat_inertia(g["inp"], dtype="f32"), oracle.kat_inertia(g["inp"], dtype="f32"))


# ---------------------------------------------------------------- goldens
@pytest.mark.parametrize("name", ["traj_single_sphere", "traj_single_cube"])
def test_single_body_trajectory_vs_reference(rb, name):
    g = load_golden(name)
    with rb.World(golden_scene(g)) as w:
        for t in range(0, 2000, 100):           # graph-replayed 100-step chunks
            w.step(100)
            q, v = w.get_state()
            assert np.array_equal(q[0], g["qpos"][t + 100]), f"{name}: qpos differs after step {t + 100}"
            assert np.array_equal(v[0], g["qvel"][t + 100]), f"{name}: qvel differs after step {t + 100}"


@pytest.mark.parametrize("name", NBODY_GOLDENS)
def test_nbody_golden_contacts_and_state(rb, name):
    g = load_golden(name)
    with rb.World(golden_scene(g)) as w:
        w.record_contacts(True)
        snaps = list(g["snap_step"])
        si = 1
        for t in range(snaps[-1]):
            w.step(1)
            if t < len(g["c_counts"]):
                cnt, par, kin, dis = w.contacts()
                a, b = g["c_off"][t], g["c_off"][t + 1]
                assert np.array_equal(cnt, g["c_counts"][t]), f"contact counts differ at step {t}"
                assert np.array_equal(par, g["c_partner"][a:b]), f"partners differ at step {t}"
                assert np.array_equal(kin, g["c_kind"][a:b]), f"kinds differ at step {t}"
                assert np.array_equal(dis, g["c_dist"][a:b]), f"dists differ at step {t}"
            if si < len(snaps) and t + 1 == snaps[si]:
                q, v = w.get_state()
                assert np.array_equal(q, g["qpos"][si]), f"qpos differs at step {t + 1}"
                assert np.array_equal(v, g["qvel"][si]), f"qvel differs at step {t + 1}"
                si += 1


# ---------------------------------------------------------------- oracle at scale
def _oracle_run(oracle, sc, steps, dtype="f64", record=False):
    osc = oracle.OracleScene(sc)
    return oracle.step(osc, sc.qpos0, sc.qvel0, steps, dtype=dtype, record=record)


@pytest.fixture
def oracle16(oracle):
    """The oracle on 16 OpenMP threads (the GPU box's host-core share)."""
    oracle.set_threads(16)
    yield oracle
    oracle.set_threads(1)


def _same(a, b):
    """Bit identity as 64-bit words (the sign of zeros counts)."""
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint64),
                                                 np.ascontiguousarray(b).view(np.uint64))


def _check_window(w, oracle, osc, q, v, first, last, tag):
    """Steps first..last (1-based, from t = 0) one launch at a time, each
    recorded: contact lists and state bit-exact with the oracle stepping
    the same state.  Returns the state after `last` and the number of
    sphere-sphere contacts seen."""
    w.record_contacts(True)
    ss = 0
    for t in range(first, last + 1):
        q, v, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
        w.step(1)
        gc, gp, gk, gd = w.contacts()
        assert np.array_equal(gc, cnt), f"{tag}: contact counts differ at step {t}"
        assert np.array_equal(gp, par) and np.array_equal(gk, kin), f"{tag}: contact partners/kinds differ at step {t}"
        assert _same(gd, dis), f"{tag}: contact distances differ at step {t}"
        gq, gv = w.get_state()
        assert _same(gq, q) and _same(gv, v), f"{tag}: state differs after step {t}"
        ss += int((kin == 16).sum())
    w.record_contacts(False)
    return q, v, ss


def test_c3_bench_windows_bit_exact(rb, oracle16):
    """The bench scene (C3, 65,536 spheres, the wide step form) from t = 0
    for 500 steps, graph-replayed between two recorded windows: the
    driver's timed window (steps 25-45: --warmup 5, K = 20) and steps
    480-500 — every recorded step's contacts and state bit-exact with the
    oracle, sphere-sphere contacts present in both windows."""
    from rbhip import scenes
    oracle = oracle16
    sc = scenes.make("c3")
    osc = oracle.OracleScene(sc)
    with rb.World(sc) as w:
        assert w.n_owned == 65536
        q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 24)
        w.step(24)
        q, v, ss1 = _check_window(w, oracle, osc, q, v, 25, 45, "c3")
        q, v = oracle.step(osc, q, v, 479 - 45)
        w.step(479 - 45)
        q, v, ss2 = _check_window(w, oracle, osc, q, v, 480, 500, "c3")
    assert ss1 > 0 and ss2 > 1000, (ss1, ss2)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,steps,every", [("c2", 2000, 500), ("c4", 400, 100), ("c5", 2000, 500)])
def test_config_long_run_bit_exact_vs_oracle(rb, oracle16, cfg, steps, every):
    """C2 and C5 (16,384 cubes) for the survey's 2,000 steps, C4 (65,536
    spheres on the incline, friction-dominated) for 400: state bit-exact
    with the oracle at every checkpoint (graph-replayed chunks; C5's replayed
    without the box kernel, rolled back where a cube pair came in range) and
    the last step's contact lists bit-exact."""
    from rbhip import scenes
    oracle = oracle16
    sc = scenes.make(cfg)
    osc = oracle.OracleScene(sc)
    q, v = sc.qpos0, sc.qvel0
    with rb.World(sc) as w:
        for t in range(0, steps - every, every):
            q, v = oracle.step(osc, q, v, every)
            w.step(every)
            gq, gv = w.get_state()
            assert _same(gq, q) and _same(gv, v), f"{cfg}: state differs after step {t + every}"
        q, v = oracle.step(osc, q, v, every - 1)
        w.step(every - 1)
        q, v, ss = _check_window(w, oracle, osc, q, v, steps, steps, cfg)
        st = w.stats()
    assert ss > 0 or cfg != "c2"          # C2 exercises sphere-sphere contacts
    if cfg == "c5":
        # chunks replayed without the box kernel (sliding cubes come within
        # bounding range now and then: those chunks were rolled back)
        assert st["box_opt_chunks"] >= 3, st


@pytest.mark.parametrize("injected", [1, 3])
def test_bucket_overflow_rolls_back_and_refits_bit_exact(rb, oracle16, monkeypatch, injected):
    """A long synchronous rb_step whose chunk overflows a bucket (a scene
    that drifted out of its fitted layout) is rolled back, the layout refitted
    to the chunk-start positions (a second overflow doubles the table) and
    the chunk replayed: bit-exact with the oracle.  The overflows are
    injected (RBHIP_DIAG_OVERFLOW): the scenes of BASELINE.json overflow a
    bucket only from genuine density — C4 after ~600 steps, when rows sliding
    at 40 m/s (0.4 m per step) pile into each other and up to 29 bodies share
    a 0.4 m cell (oracle-measured; 30 fit a bucket), which stays an error."""
    from rbhip import scenes
    monkeypatch.setenv("RBHIP_DIAG_OVERFLOW", str(injected))
    sc = scenes.flat_spheres(160, 160, seed=3)          # 25,600: the wide form's linear layout
    with rb.World(sc) as w:
        h0 = w.stats()["buckets"]
        w.step(300)
        q, v = w.get_state()
        st = w.stats()
    q1, v1 = oracle16.step(oracle16.OracleScene(sc), sc.qpos0, sc.qvel0, 300)
    assert _same(q, q1) and _same(v, v1)
    assert st["refits"] == injected, st
    assert st["table_grows"] == injected - 1 and st["buckets"] == h0 << (injected - 1), st


@pytest.mark.parametrize("form,env", [("coop", {}), ("wide", {"RBHIP_COOP_MAX_BODIES": "0"}),
                                      ("wide_plain", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_HELP": "0"}),
                                      ("one", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_MAX_BODIES": "0"})])
def test_crowded_cells_spill_bit_exact(rb, oracle16, monkeypatch, form, env):
    """Hundreds of bodies in one broadphase cell (scenes.crowded_cells: a
    r 1.0 sphere sets 4-m cells, 400 spheres of r 0.05 pile up in one): the
    ids past each bucket's 30 slots spill into the table's spill list, which
    every search form reads for a full bucket — contacts (recorded steps) and
    state bit-exact with the oracle, whose broadphase has no capacity."""
    from rbhip import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = scenes.crowded_cells()
    cells = np.floor(sc.qpos0[:-1, :3] / (4.0 * 1.0 * 1.001)).astype(np.int64)
    assert np.unique(cells, axis=0, return_counts=True)[1].max() > 30
    osc = oracle16.OracleScene(sc)
    q, v = sc.qpos0, sc.qvel0
    with rb.World(sc) as w:
        for t in (99, 99):
            q, v = oracle16.step(osc, q, v, t)
            w.step(t)
            w.record_contacts(True)
            q, v, (cnt, par, kin, dis) = oracle16.step(osc, q, v, 1, record=True)
            w.step(1)
            gc, gp, gk, gd = w.contacts()
            w.record_contacts(False)
            assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
            assert _same(gd, dis)
            gq, gv = w.get_state()
            assert _same(gq, q) and _same(gv, v)
    assert cnt.sum() > 100                            # the pile is in contact


@pytest.mark.timeout(900)
def test_c4_2000_steps_bit_exact(rb, oracle16):
    """configs[3]'s scene for 2,000 steps from t = 0 with the default world:
    after ~550 steps the sliding rows pile into each other (up to 28 sphere
    partners: a guarded rb_step chunk rolls back and raises max_partners to
    32; up to 29+ bodies in a cell: full buckets spill) — bit-exact with the
    oracle."""
    from rbhip import scenes
    sc = scenes.make("c4")
    with rb.World(sc) as w:
        for _ in range(4):
            w.step(500)
        q, v = w.get_state()
        st = w.stats()
    q1, v1 = oracle16.step(oracle16.OracleScene(sc, max_partners=32), sc.qpos0, sc.qvel0, 2000)
    assert _same(q, q1) and _same(v, v1)
    assert st["max_partners"] == 32, st


def test_c3_one_step_parity_from_evolved_state(rb, oracle):
    """65,536 spheres: 30 oracle steps, then one GPU step from that state vs
    one oracle step (contacts and state bit-exact)."""
    from rbhip import scenes
    sc = scenes.make("c3")
    osc = oracle.OracleScene(sc)
    q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 30)
    q1, v1, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
    with rb.World(sc.with_(qpos0=q, qvel0=v)) as w:
        w.record_contacts(True)
        w.step(1)
        gq, gv = w.get_state()
        gc, gp, gk, gd = w.contacts()
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
    assert np.array_equal(gq, q1) and np.array_equal(gv, v1)


def test_large_scene_steps_parity(rb, oracle, monkeypatch):
    """409,600 spheres (above 300k the broadphase groups buckets by 2x2x2
    super-cell): 70 GPU steps, then one recorded step, vs the oracle (16
    threads) — contacts and state bit-exact, in the tile form (the default
    above 65,536 bodies) and in the hashed-cell forms
    (RBHIP_TILE=0)."""
    from rbhip import scenes
    # grid spacing 0.19 < 2r: neighbours collide once they land
    sc = scenes.flat_spheres(640, 640, seed=5, spacing=0.19)
    osc = oracle.OracleScene(sc)
    oracle.set_threads(16)
    try:
        q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 70)
        q1, v1, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
    finally:
        oracle.set_threads(1)
    for tile in ("-1", "0"):
        monkeypatch.setenv("RBHIP_TILE", tile)
        with rb.World(sc) as w:
            w.step(70)
            gq, gv = w.get_state()
            assert np.array_equal(gq, q) and np.array_equal(gv, v), f"RBHIP_TILE={tile}"
            w.record_contacts(True)
            w.step(1)
            gq, gv = w.get_state()
            gc, gp, gk, gd = w.contacts()
            st = w.stats()
        assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin), f"RBHIP_TILE={tile}"
        assert np.array_equal(gq, q1) and np.array_equal(gv, v1), f"RBHIP_TILE={tile}"
        assert (st["form"] == 5 and st["tile_steps"] == 71) == (tile == "-1"), st
    assert (kin == 16).sum() > 1000


def test_f32_bit_exact_vs_f32_restatement(rb, oracle):
    from rbhip import scenes
    sc = scenes.make("c2")
    q0, v0 = _oracle_run(oracle, sc, 150, dtype="f32")
    with rb.World(sc, dtype="f32") as w:
        w.step(150)
        q, v = w.get_state()
    assert np.array_equal(q, q0) and np.array_equal(v, v0)


@pytest.mark.parametrize("horizon,max_flip_frac,med_rel,p999_d,max_d",
                         [(1, 1e-3, 1e-6, 1e-4, 1e-3), (10, 5e-3, 1e-6, 1e-3, None)])
def test_f32_vs_f64_tolerance_sweep(rb, oracle, horizon, max_flip_frac, med_rel, p999_d, max_d):
    """C3 fp32-vs-fp64 sweep (SURVEY §8d, §7 hard part 5): from the same
    evolved fp64 state, `horizon` steps in each precision — contact flips
    (pairs present in one list only, last step) and the state error.
    Asserted at 1 step (flips <= 0.1 %, max |dpos| < 1 mm) and 10 steps
    (flips <= 0.5 %, median relative error < 1e-6, 99.9th percentile of
    |dpos| < 1 mm; measured on MI355X: 6 flips of 3,662 contacts, median
    1.0e-7 — a flipped contact sends its bodies elsewhere, 5 cm after 10
    steps, so the maximum is reported, not bounded).  The 100- and 200-step
    divergence from t = 0 is bench.py's fp32 line
    (profiles/r03/bench_c3_f32.json)."""
    from rbhip import scenes
    sc = scenes.make("c3")
    q, v = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 30)
    res = {}
    for dt in ("f64", "f32"):
        with rb.World(sc.with_(qpos0=q, qvel0=v), dtype=dt) as w:
            if horizon > 1:
                w.step(horizon - 1)
            w.record_contacts(True)
            w.step(1)
            qq, vv = w.get_state()
            cnt, par, kin, dis = w.contacts()
        body = np.repeat(np.arange(sc.n), cnt)
        res[dt] = (qq, vv, set(zip(body.tolist(), par.tolist())))
    flips = len(res["f64"][2] ^ res["f32"][2])
    ncon = len(res["f64"][2])
    d = np.abs(res["f32"][0][:, :3] - res["f64"][0][:, :3])
    rel = d / (1.0 + np.abs(res["f64"][0][:, :3]))
    dn = np.linalg.norm(d, axis=1)
    print(f"\nC3 fp32 vs fp64, {horizon} step(s) from step 30: {ncon} contacts, {flips} flips, "
          f"median rel dpos {np.median(rel):.2e}, p99.9 |dpos| {np.quantile(dn, 0.999):.2e}, max |dpos| {d.max():.2e}")
    assert ncon > 1000 and flips <= max(2, int(ncon * max_flip_frac))
    assert np.median(rel) < med_rel and np.quantile(dn, 0.999) < p999_d
    if max_d is not None:
        assert d.max() < max_d


@pytest.mark.parametrize("env", [{}, {"RBHIP_COOP_MAX_BODIES": "0"}, {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_HELP": "0"}],
                         ids=["coop_help", "wide_help", "wide_plain"])
def test_xfrc_applied_matches_oracle(rb, oracle, monkeypatch, env):
    """Applied forces (collision.py:66-70): the helper-wave forms leave them
    to the body lanes."""
    from rbhip import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = scenes.flat_spheres(16, 16, seed=5)
    rng = np.random.default_rng(0)
    xf = rng.normal(0, 0.5, (sc.n, 6))
    osc = oracle.OracleScene(sc)
    q0, v0 = oracle.step(osc, sc.qpos0, sc.qvel0, 80, xfrc=xf)
    with rb.World(sc) as w:
        w.set_xfrc(xf)
        w.step(80)
        q, v = w.get_state()
    assert np.array_equal(q, q0) and np.array_equal(v, v0)


# ---------------------------------------------------------------- determinism / sharding
def test_graph_equals_single_launches_and_reruns(rb):
    from rbhip import scenes
    sc = scenes.make("c2")
    res = []
    for mode in ("graph", "single", "graph"):
        with rb.World(sc) as w:
            if mode == "graph":
                w.step(200)
            else:
                for _ in range(200):
                    w.step_async(1)
                w.sync()
            res.append(w.get_state())
    for q, v in res[1:]:
        assert np.array_equal(q, res[0][0]) and np.array_equal(v, res[0][1])


@pytest.mark.parametrize("P,scene,steps", [(2, "flat800", 120), (3, "flat800", 120), (4, "flat800", 120),
                                           (8, "c4", 240), (2, "boxpile", 400), (3, "boxpile", 400)])
def test_shard_invariance_in_process(rb, P, scene, steps):
    """P body-range shards on one device, positions (and in box worlds the
    orientations) exchanged by device copies between their replicated
    buffers: bit-identical (uint64 words) to one world, and the last step's
    contact lists equal.  (8, "c4") is BASELINE configs[3] as the 8-GPU run
    shards it: 65,536 spheres on the incline, 8,192 per rank (the body loop
    of multi_sphere_bounce.py:46-90 split by body-id range).  "boxpile":
    cube columns with sphere caps, shards meeting along a row of columns
    (box-box, edge and sphere-box contacts across the seam)."""
    import torch
    from rbhip import scenes
    from rbhip.shard import wrap_gpos, wrap_gquat
    kw = {}
    if scene == "flat800":
        sc = scenes.flat_spheres(32, 25, seed=7)       # 800: not a multiple of 3
    elif scene == "boxpile":
        sc, kw = scenes.box_pile(6, 6, 3, seed=0), {"max_partners": 32}
    else:
        sc = scenes.make(scene)
    with rb.World(sc, **kw) as ref:
        ref.step(steps - 1)
        ref.record_contacts(True)
        ref.step(1)
        rq, rv = ref.get_state()
        rc, rp, rk, rd = ref.contacts()
    worlds = [rb.World(sc, rank=r, world_size=P, **kw) for r in range(P)]
    for s in range(steps):
        if s == steps - 1:
            for w in worlds:
                w.record_contacts(True)
        for w in worlds:
            w.shard_step()
        for w in worlds:
            w.sync()
        for wrap in (wrap_gpos, wrap_gquat):
            bufs = [wrap(w, torch) for w in worlds]      # the buffers alternate per step
            n = bufs[0][1]
            if bufs[0][0] is None:                       # sphere worlds: no orientations
                continue
            for r, (buf, _) in enumerate(bufs):
                for o, (obuf, _) in enumerate(bufs):
                    if o != r:
                        buf[o * n:(o + 1) * n].copy_(obuf[o * n:(o + 1) * n])
        torch.cuda.synchronize()
        for w in worlds:
            w.shard_exchange_done()
    q = np.zeros((sc.n, 7))
    v = np.zeros((sc.n, 6))
    cnt, par, kin, dis = [], [], [], []
    for w in worlds:
        w.get_state(q, v)
        c, pa, k, d = w.contacts()
        cnt.append(c); par.append(pa); kin.append(k); dis.append(d)
        w.close()
    assert np.array_equal(q.view(np.uint64), rq.view(np.uint64)) and np.array_equal(v.view(np.uint64), rv.view(np.uint64))
    assert np.array_equal(np.concatenate(cnt), rc) and np.array_equal(np.concatenate(par), rp)
    assert np.array_equal(np.concatenate(kin), rk)
    assert np.array_equal(np.concatenate(dis).view(np.uint64), rd.view(np.uint64))


# ---------------------------------------------------------------- loud failures
def test_bucket_or_partner_overflow_is_an_error(rb):
    from rbhip import scenes
    sc = scenes.flat_spheres(6, 6, seed=0)
    q = sc.qpos0.copy()
    q[:, 0:3] = [0.0, 0.0, 1.0]                       # 36 spheres at one point
    with rb.World(sc.with_(qpos0=q)) as w:
        with pytest.raises(rb.RbError, match="EOVERFLOW"):
            w.step(1)


def test_nonfinite_position_is_an_error(rb):
    from rbhip import scenes
    sc = scenes.flat_spheres(4, 4, seed=0)
    q = sc.qpos0.copy()
    q[3, 2] = np.nan
    with rb.World(sc.with_(qpos0=q)) as w:
        with pytest.raises(rb.RbError, match="EDOM"):
            w.step(1)


def test_error_word_around_graph_runs(rb):
    """Every captured graph ends by publishing the error word to pinned host
    memory, so rb_sync after a graph only synchronises; an error-writing
    launch enqueued after the graph (here an eager single step) must make
    rb_sync publish again — and an error inside a graph run is reported by
    the graph's own publish.  No stale bits after an error is cleared."""
    from rbhip import scenes
    sc = scenes.flat_spheres(8, 8, seed=0)
    bad = sc.qpos0.copy()
    bad[3, 2] = np.nan
    with rb.World(sc) as w:
        w.step(20)
        w.sync()
        w.set_state(bad, sc.qvel0)
        w.step_async(1)                                  # eager, after the graph
        with pytest.raises(rb.RbError, match="EDOM"):
            w.sync()
        w.set_state(sc.qpos0, sc.qvel0)
        w.step(20)
        w.sync()
        w.set_state(bad, sc.qvel0)
        with pytest.raises(rb.RbError, match="EDOM"):
            w.step(20)                                   # raised inside the graph
        w.set_state(sc.qpos0, sc.qvel0)
        w.step(20)
        w.sync()
        w.step(1)
        w.sync()


def test_box_pair_across_shards_is_solved(rb):
    """Two cubes within bounding range, one per shard: the exchange carries
    their orientations (rb_gquat_buffer), so the pair is solved exactly as
    in one world (this was RB_EUNSUPPORTED before round 3)."""
    import torch
    from rbhip import scenes
    from rbhip.shard import wrap_gpos, wrap_gquat
    sc = scenes.incline_cubes(2, 1, seed=0, spacing=0.5)
    with rb.World(sc) as ref:
        ref.step(60)
        rq, rv = ref.get_state()
    worlds = [rb.World(sc, rank=r, world_size=2) for r in range(2)]
    for _ in range(60):
        for w in worlds:
            w.shard_step()
        for w in worlds:
            w.sync()
        for wrap in (wrap_gpos, wrap_gquat):
            (b0, n), (b1, _) = wrap(worlds[0], torch), wrap(worlds[1], torch)
            b0[n:2 * n].copy_(b1[n:2 * n])
            b1[0:n].copy_(b0[0:n])
        torch.cuda.synchronize()
        for w in worlds:
            w.shard_exchange_done()
    q = np.zeros((sc.n, 7))
    v = np.zeros((sc.n, 6))
    for w in worlds:
        w.get_state(q, v)
        w.close()
    assert np.array_equal(q.view(np.uint64), rq.view(np.uint64)) and np.array_equal(v.view(np.uint64), rv.view(np.uint64))


def test_graph_cache_stays_bounded(rb):
    """stepping with many different (K, dt, ...) keys keeps at
    most GRAPH_CACHE_MAX (32) captured graphs alive (both parities of a key
    are captured together; the least recently used are destroyed), and a
    key evicted earlier is captured again when it comes back."""
    from rbhip import scenes
    with rb.World(scenes.flat_spheres(8, 8, seed=1)) as w:
        seen = []
        for k in range(40):
            w.step(2 + k % 3, dt=0.01 + 1e-4 * k)
            seen.append(w.stats()["graphs"])
        w.step(2, dt=0.01)                        # the first key again
        seen.append(w.stats()["graphs"])
    assert max(seen) <= 32 and seen[-1] <= 32, seen
    assert seen[0] == 2 and seen[15] == 32, seen  # two entries per key until the cap


def test_empty_world_and_idle_shards(rb):
    """Edge cases: a world with no bodies is refused (RB_EINVAL, "n_bodies
    out of range": nothing to step, and no device buffers of size 0); a
    3-body scene over 4 shards (rank 3 owns no body) matches one world."""
    import torch
    from rbhip import scenes
    from rbhip.shard import wrap_gpos
    sc0 = scenes.flat_spheres(2, 2).with_(kind=np.zeros(0, np.int32), mass=np.zeros(0), inertia=np.zeros((0, 3)),
                                         size=np.zeros((0, 3)), qpos0=np.zeros((0, 7)), qvel0=np.zeros((0, 6)))
    with pytest.raises(rb.RbError, match="EINVAL"):
        rb.World(sc0)
    sc = scenes.multi_sphere4().with_()
    sc = sc.with_(kind=sc.kind[:3], mass=sc.mass[:3], inertia=sc.inertia[:3], size=sc.size[:3],
                  qpos0=sc.qpos0[:3], qvel0=sc.qvel0[:3], names=None)
    with rb.World(sc) as ref:
        ref.step(200)
        rq, rv = ref.get_state()
    worlds = [rb.World(sc, rank=r, world_size=4) for r in range(4)]
    assert [w.n_owned for w in worlds] == [1, 1, 1, 0]
    for _ in range(200):
        for w in worlds:
            w.shard_step()
        for w in worlds:
            w.sync()
        bufs = [wrap_gpos(w, torch) for w in worlds]
        n = bufs[0][1]
        for r, (buf, _) in enumerate(bufs):
            for o, (obuf, _) in enumerate(bufs):
                if o != r:
                    buf[o * n:(o + 1) * n].copy_(obuf[o * n:(o + 1) * n])
        torch.cuda.synchronize()
        for w in worlds:
            w.shard_exchange_done()
    q = np.zeros((3, 7))
    v = np.zeros((3, 6))
    for w in worlds:
        w.get_state(q, v)
        w.close()
    assert np.array_equal(q.view(np.uint64), rq.view(np.uint64)) and np.array_equal(v.view(np.uint64), rv.view(np.uint64))


def test_kernel_timing_reports_launches(rb):
    from rbhip import scenes
    with rb.World(scenes.make("c2")) as w:
        w.kernel_timing(True)
        w.step(20)
        avg, n = w.kernel_timing(False)
    assert n == 20 and 0 < avg < 50.0
    assert C.sizeof(C.c_double) == 8 and time.time() > 0


def test_wide_form_on_contact_rich_scene_bit_exact(rb, oracle, monkeypatch):
    """The wide one-lane form (32-byte bucket heads, LDS candidate list,
    state loads under the search) on C2, 300 steps with many sphere-sphere
    contacts and buckets of several bodies: contacts and state bit-exact
    with the oracle."""
    from rbhip import scenes
    monkeypatch.setenv("RBHIP_COOP_MAX_BODIES", "0")        # 4,096 bodies through the wide form
    sc = scenes.make("c2")
    q0, v0, (cnt, par, kin, dis) = _oracle_run(oracle, sc, 300, record=True)
    with rb.World(sc) as w:
        w.step(299)
        w.record_contacts(True)
        w.step(1)
        q, v = w.get_state()
        gc, gp, gk, gd = w.contacts()
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
    assert np.array_equal(q, q0) and np.array_equal(v, v0)
    assert (kin == 16).sum() > 100


def test_wide_form_buckets_past_the_head_bit_exact(rb, oracle, monkeypatch):
    """The wide form's rare path: buckets of 7+ bodies, whose ids past the
    32-byte head (6 ids) are read from the bucket's further lines.  A flat
    grid at spacing 0.15 puts up to 9 landed spheres in one 0.4-m cell; 120
    steps, then one recorded step, contacts and state bit-exact with the
    oracle, and the scene is checked to hold such cells."""
    from rbhip import scenes
    monkeypatch.setenv("RBHIP_COOP_MAX_BODIES", "0")
    sc = scenes.flat_spheres(33, 31, seed=5, spacing=0.15)
    q0, v0, (cnt, par, kin, dis) = _oracle_run(oracle, sc, 121, record=True)
    with rb.World(sc) as w:
        w.step(120)
        w.record_contacts(True)
        w.step(1)
        q, v = w.get_state()
        gc, gp, gk, gd = w.contacts()
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
    assert np.array_equal(gd, dis)
    assert np.array_equal(q, q0) and np.array_equal(v, v0)
    # cells (2 x 2 r = 0.4 m) holding 7+ bodies: the path is exercised
    cells = np.floor(q0.reshape(-1, 7)[:, :3] / 0.4).astype(np.int64)
    _, per_cell = np.unique(cells, axis=0, return_counts=True)
    assert per_cell.max() >= 7


@pytest.mark.parametrize("form,env", [
    ("coop", {}),
    ("coop_help", {"RBHIP_HELP_MAX_BODIES": "100000"}),
    ("wide", {"RBHIP_COOP_MAX_BODIES": "0"}),
    ("wide_plain", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_HELP": "0"}),
    ("one", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_MAX_BODIES": "0"}),
    ("split", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_MAX_BODIES": "0", "RBHIP_SPLIT": "1"}),
])
def test_ragged_scene_every_step_form_bit_exact(rb, oracle, monkeypatch, form, env):
    """A body count that fills no workgroup evenly (37 x 29 = 1,073; the last
    wave is partial) on a packed grid (spacing 0.19 < 2r: neighbours collide
    once they land), through each step form the library can pick: 120
    steps, then one recorded step, contacts and state bit-exact with the
    oracle."""
    from rbhip import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = scenes.flat_spheres(37, 29, seed=3, spacing=0.19)
    assert sc.n % 64 != 0
    q0, v0, (cnt, par, kin, dis) = _oracle_run(oracle, sc, 121, record=True)
    with rb.World(sc) as w:
        w.step(120)
        w.record_contacts(True)
        w.step(1)
        q, v = w.get_state()
        gc, gp, gk, gd = w.contacts()
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
    assert np.array_equal(gd, dis)
    assert np.array_equal(q, q0) and np.array_equal(v, v0)
    assert (kin == 16).sum() > 50                      # sphere-sphere contacts in the recorded step
