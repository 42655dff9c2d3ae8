"""The cell-ordered tile form (csrc/rb_tiles.hip) against the
oracle and the hashed-cell forms, through the C-ABI.

The form is the default for eligible worlds of > 65,536 bodies
(RBHIP_TILE=-1, auto); these tests force it (RBHIP_TILE=1 at world
creation) or turn it off (0) on smaller scenes.  Bar: fp64 bit-exact
(contacts and state, compared as uint64 words) — the tile form only changes
where a body's candidates come from, not the arithmetic or the contact
order.  Its failure paths (a full bin, window or far list; too many partners)
roll the run back and replay it with the hashed forms, which must leave the
same bits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


@pytest.fixture
def oracle16(oracle):
    oracle.set_threads(16)
    yield oracle
    oracle.set_threads(1)


def _same(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint64),
                                                 np.ascontiguousarray(b).view(np.uint64))


def _world(rb, monkeypatch, sc, tile, **kw):
    monkeypatch.setenv("RBHIP_TILE", "1" if tile else "0")
    w = rb.World(sc, **kw)
    monkeypatch.delenv("RBHIP_TILE")
    return w


def test_tile_c3_from_rest_vs_oracle(rb, oracle16, monkeypatch):
    """configs[2] (65,536 spheres) in tile slots: 24 graph-replayed steps from
    t = 0, then steps 25-27 one launch each with contacts recorded — state
    and contact lists bit-exact with the oracle; the steps ran in the tile
    form (no roll-back)."""
    from rbhip import scenes
    sc = scenes.make("c3")
    osc = oracle16.OracleScene(sc)
    with _world(rb, monkeypatch, sc, True) as w:
        q, v = oracle16.step(osc, sc.qpos0, sc.qvel0, 24)
        w.step(24)
        gq, gv = w.get_state()
        assert _same(gq, q) and _same(gv, v), "state differs after step 24"
        w.record_contacts(True)
        for t in range(25, 28):
            q, v, (cnt, par, kin, dis) = oracle16.step(osc, q, v, 1, record=True)
            w.step(1)
            gc, gp, gk, gd = w.contacts()
            assert np.array_equal(gc, cnt), f"contact counts differ at step {t}"
            assert np.array_equal(gp, par) and np.array_equal(gk, kin), f"partners differ at step {t}"
            assert _same(gd, dis), f"contact distances differ at step {t}"
            gq, gv = w.get_state()
            assert _same(gq, q) and _same(gv, v), f"state differs after step {t}"
        st = w.stats()
    assert st["form"] == 5 and st["tile_steps"] == 27 and st["tile_rollbacks"] == 0, st


def test_tile_async_chain_matches_hashed(rb, monkeypatch):
    """Tile runs chain without a sync between them (their checks wait for
    the next sync point): 5 + 20 + 20 + 1 + 1 steps enqueued back to back,
    bit-identical to the hashed forms after each sync."""
    from rbhip import scenes
    sc = scenes.flat_spheres(96, 96, seed=4)
    wt = _world(rb, monkeypatch, sc, True)
    wh = _world(rb, monkeypatch, sc, False)
    try:
        for chunk in ([5, 20, 20], [1, 1], [50]):
            for n in chunk:
                wt.step_async(n)
                wh.step_async(n)
            wt.sync()
            wh.sync()
            qt, vt = wt.get_state()
            qh, vh = wh.get_state()
            assert _same(qt, qh) and _same(vt, vh), f"differs after chunk {chunk}"
        st = wt.stats()
        assert st["form"] == 5 and st["tile_steps"] == 97 and st["tile_runs"] >= 6, st
        assert wh.stats()["form"] != 5
    finally:
        wt.close()
        wh.close()


def test_tile_far_movers_vs_oracle(rb, oracle16, monkeypatch):
    """Bodies thrown across several columns per step go through the far
    list (they leave their tile's ring): bit-exact with the oracle."""
    from rbhip import scenes
    sc = scenes.flat_spheres(64, 64, seed=5)
    rng = np.random.default_rng(7)
    fast = rng.choice(sc.n, 24, replace=False)
    qvel = sc.qvel0.copy()
    qvel[fast, 0] = rng.uniform(-400.0, 400.0, fast.size)   # up to ~0.8 m (2+ columns) per step
    qvel[fast, 1] = rng.uniform(-400.0, 400.0, fast.size)
    osc = oracle16.OracleScene(sc)
    with _world(rb, monkeypatch, sc, True) as w:
        w.set_state(sc.qpos0, qvel)
        w.step(40)
        gq, gv = w.get_state()
        st = w.stats()
    q, v = oracle16.step(osc, sc.qpos0, qvel, 40)
    assert _same(gq, q) and _same(gv, v)
    assert st["tile_steps"] + 40 * st["tile_rollbacks"] >= 40, st


def test_tile_rollback_replays_bit_exact(rb, oracle16, monkeypatch):
    """configs[3]'s incline piles up after ~550 steps: a slot then holds more
    bodies than its workgroup has lanes (TILE_WHY_CAP), the run rolls back
    and is replayed with the hashed forms, and the layout is refitted — the
    state after 700 steps bit-exact with the oracle."""
    from rbhip import scenes
    sc = scenes.make("c4")
    with _world(rb, monkeypatch, sc, True, max_partners=32) as w:
        for _ in range(14):
            w.step_async(50)
        w.sync()
        gq, gv = w.get_state()
        st = w.stats()
    q, v = oracle16.step(oracle16.OracleScene(sc, max_partners=32), sc.qpos0, sc.qvel0, 700)
    assert _same(gq, q) and _same(gv, v)
    assert st["tile_rollbacks"] >= 1 and st["tile_why"] & 1, st


def test_tile_crowded_column_rolls_back_bit_exact(rb, oracle16, monkeypatch):
    """A column past a slot's 128 lanes (scenes.crowded_cells: ~400 spheres
    in one 4-m column) raises TILE_WHY_CAP on the first step: the run rolls
    back and is replayed with the hashed forms — state bit-exact with the
    oracle, the roll-back counted."""
    from rbhip import scenes
    sc = scenes.crowded_cells()
    osc = oracle16.OracleScene(sc)
    with _world(rb, monkeypatch, sc, True) as w:
        w.step_async(20)
        w.step_async(20)
        w.sync()
        gq, gv = w.get_state()
        st = w.stats()
    q, v = oracle16.step(osc, sc.qpos0, sc.qvel0, 40)
    assert _same(gq, q) and _same(gv, v)
    assert st["tile_rollbacks"] >= 1 and st["tile_why"] & (1 | 2), st


def test_tile_form_declines_what_it_cannot_step(rb, monkeypatch):
    """Worlds outside the tile form's reach step with the hashed forms even
    with RBHIP_TILE=1: box bodies, applied forces."""
    from rbhip import scenes
    sc = scenes.incline_cubes(8, 8, seed=1)
    with _world(rb, monkeypatch, sc, True) as w:
        w.step(3)
        assert w.stats()["form"] != 5
    sc = scenes.flat_spheres(40, 40, seed=2)
    with _world(rb, monkeypatch, sc, True) as w:
        xf = np.zeros((sc.n, 6))
        xf[:, 0] = 1.0
        w.set_xfrc(xf)
        w.step(3)
        st = w.stats()
        assert st["form"] != 5 and st["tile_steps"] == 0, st


def test_tile_auto_mode_retires_after_rollback(rb, oracle16, monkeypatch):
    """Auto mode (the default; RBHIP_TILE_MIN_BODIES lowered so the small
    crowded scene qualifies): the first roll-back retires the tile form for
    the world (its bins freed) — every later run steps hashed, no second
    roll-back — and the state stays bit-exact with the oracle; an
    rb_set_state of a new state re-arms the auto mode."""
    from rbhip import scenes
    sc = scenes.crowded_cells()
    osc = oracle16.OracleScene(sc)
    monkeypatch.setenv("RBHIP_TILE_MIN_BODIES", "1")
    monkeypatch.delenv("RBHIP_TILE", raising=False)
    with rb.World(sc) as w:
        monkeypatch.delenv("RBHIP_TILE_MIN_BODIES")
        for _ in range(6):
            w.step_async(10)
        w.sync()
        st0 = w.stats()
        w.step(20)
        gq, gv = w.get_state()
        st = w.stats()
        w.set_state(sc.qpos0, sc.qvel0)
        st2 = w.stats()
    q, v = oracle16.step(osc, sc.qpos0, sc.qvel0, 80)
    assert _same(gq, q) and _same(gv, v)
    assert st0["tile_rollbacks"] == 1 and st["tile_rollbacks"] == 1, (st0, st)
    assert st["form"] != 5 and st["tile_on"] == 0, st
    assert st2["tile_on"] == 1, st2


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_auto_threshold_and_default_form_vs_oracle(rb, oracle16, monkeypatch, dtype):
    """The default (auto) mode: 65,536 spheres (C3's size) step hashed,
    65,792 (256 x 257) in the tile form — from rest, 150 steps bit-exact
    with the oracle in both precisions (fp32 against the fp32 restatement),
    then one recorded step with identical contact lists."""
    from rbhip import scenes
    monkeypatch.delenv("RBHIP_TILE", raising=False)
    monkeypatch.delenv("RBHIP_TILE_MIN_BODIES", raising=False)
    with rb.World(scenes.flat_spheres(256, 256, seed=3), dtype=dtype) as w:
        w.step(4)
        assert w.stats()["form"] != 5
    sc = scenes.flat_spheres(256, 257, seed=3)
    osc = oracle16.OracleScene(sc)
    q, v = oracle16.step(osc, sc.qpos0, sc.qvel0, 150, dtype=dtype)
    q1, v1, (cnt, par, kin, dis) = oracle16.step(osc, q, v, 1, dtype=dtype, record=True)
    with rb.World(sc, dtype=dtype) as w:
        w.step(150)
        gq, gv = w.get_state()
        assert _same(gq, q) and _same(gv, v)
        w.record_contacts(True)
        w.step(1)
        gq, gv = w.get_state()
        gc, gp, gk, gd = w.contacts()
        st = w.stats()
    assert st["form"] == 5 and st["tile_steps"] == 151 and st["tile_rollbacks"] == 0, st
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)
    assert _same(gd, dis) and _same(gq, q1) and _same(gv, v1)
    assert cnt.sum() > 0


def test_auto_mode_declines_a_spread_scene(rb, oracle16, monkeypatch):
    """Auto mode on a scene spread far (65,792 spheres plus one 2 km away: the
    tile grid folds onto its most slots, ~5 KB of bins per body) declines
    the tile form and steps hashed — bit-exact with the oracle; forced
    (RBHIP_TILE=1) the same scene steps in tile slots, bit-exact too."""
    from rbhip import scenes
    sc = scenes.flat_spheres(256, 257, seed=3)
    q0 = sc.qpos0.copy()
    q0[-1, 0] += 2000.0
    sc = sc.with_(qpos0=q0)
    q, v = oracle16.step(oracle16.OracleScene(sc), sc.qpos0, sc.qvel0, 30)
    monkeypatch.delenv("RBHIP_TILE", raising=False)
    with rb.World(sc) as w:
        w.step(30)
        gq, gv = w.get_state()
        st = w.stats()
    assert _same(gq, q) and _same(gv, v)
    assert st["form"] != 5 and st["tile_steps"] == 0 and st["tile_on"] == 0, st
    with _world(rb, monkeypatch, sc, True) as w:
        w.step(30)
        gq, gv = w.get_state()
        st = w.stats()
    assert _same(gq, q) and _same(gv, v)
    assert st["form"] == 5 and st["tile_steps"] == 30, st


@pytest.mark.timeout(600)
def test_tile_c3_2000_steps_vs_oracle(rb, oracle16, monkeypatch):
    """The tile form forced onto configs[2] (65,536 spheres) for 2,000 steps
    from rest, in async runs of 500 (the spheres land, bounce and settle):
    bit-exact with the oracle, every step in tile slots."""
    from rbhip import scenes
    sc = scenes.make("c3")
    with _world(rb, monkeypatch, sc, True) as w:
        for _ in range(4):
            w.step_async(500)
        w.sync()
        gq, gv = w.get_state()
        st = w.stats()
    q, v = oracle16.step(oracle16.OracleScene(sc), sc.qpos0, sc.qvel0, 2000)
    assert _same(gq, q) and _same(gv, v)
    assert st["tile_steps"] == 2000 and st["tile_rollbacks"] == 0, st


@pytest.mark.timeout(600)
def test_tile_default_one_million_vs_oracle(rb, oracle16, monkeypatch):
    """1,048,576 spheres (1024 x 1024, grid spacing 0.19 < 2r: neighbours
    collide on landing) in the default (auto) mode — the tile form with the
    3-wave kernel (12k+ slots) — 80 steps, then one recorded step: state and
    contact lists bit-exact with the oracle."""
    from rbhip import scenes
    monkeypatch.delenv("RBHIP_TILE", raising=False)
    sc = scenes.flat_spheres(1024, 1024, seed=6, spacing=0.19)
    osc = oracle16.OracleScene(sc)
    q, v = oracle16.step(osc, sc.qpos0, sc.qvel0, 80)
    q1, v1, (cnt, par, kin, dis) = oracle16.step(osc, q, v, 1, record=True)
    with rb.World(sc) as w:
        w.step(80)
        gq, gv = w.get_state()
        assert _same(gq, q) and _same(gv, v)
        w.record_contacts(True)
        w.step(1)
        gq, gv = w.get_state()
        gc, gp, gk, gd = w.contacts()
        st = w.stats()
    assert st["form"] == 5 and st["tile_steps"] == 81 and st["tile_slots"] > 1024, st
    bad = np.flatnonzero(gc != cnt)
    go, oo = np.concatenate([[0], np.cumsum(gc)]), np.concatenate([[0], np.cumsum(cnt)])
    detail = [(int(b), gp[go[b]:go[b + 1]].tolist(), gk[go[b]:go[b + 1]].tolist(),
               par[oo[b]:oo[b + 1]].tolist(), kin[oo[b]:oo[b + 1]].tolist()) for b in bad[:4]]
    assert not bad.size, f"contact counts differ at {bad.size} bodies (state@81 same: " \
                         f"{_same(gq, q1) and _same(gv, v1)}): {detail}"
    assert np.array_equal(gp, par) and np.array_equal(gk, kin), np.flatnonzero((gp != par) | (gk != kin))[:8]
    assert _same(gd, dis) and _same(gq, q1) and _same(gv, v1)
    assert (kin == 16).sum() > 1000
