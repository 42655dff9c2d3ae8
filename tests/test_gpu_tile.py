"""K-step tile blocks (rb_tile.hip) against the oracle.

The tile path steps a tile plus a ghost band up to K reference steps per
launch and commits a block only when it is provably identical to single
steps.  Bar: fp64 (and fp32 against the fp32 restatement) bit-exact, state
compared as uint64 words, after runs that commit many blocks and redo some;
the counters prove the tile path actually ran (rb_world_stats)."""
import numpy as np
import pytest

from rbhip import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


def words(a):
    return np.ascontiguousarray(a).view(np.uint64 if a.dtype == np.float64 else np.uint32)


def assert_same(q, v, q1, v1, what):
    bad = np.flatnonzero(~(np.all(words(q) == words(q1), axis=1) & np.all(words(v) == words(v1), axis=1)))
    assert bad.size == 0, f"{what}: {bad.size} bodies differ, first {bad[:8].tolist()}"


def run_tile(rb, sc, steps, dtype="f64", chunks=1, **cfg):
    with rb.World(sc, dtype=dtype) as w:
        w.tile_config(1, **cfg)
        for _ in range(chunks):
            w.step(steps)
        q, v = w.get_state()
        return q, v, w.stats()


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_tile_blocks_bit_exact_vs_oracle(rb, oracle, cfg):
    """65,536 spheres from t = 0 (the bench scene and the incline), 120 steps
    in blocks of up to 8, against the 16-thread oracle."""
    sc = scenes.make(cfg)
    q, v, st = run_tile(rb, sc, 120)
    assert st["tile_steps"] == 120 and st["tile_blocks"] >= 15 and st["tile_fallback"] == 0, st
    oracle.set_threads(16)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 120)
    assert_same(q, v, q1, v1, f"{cfg} tile blocks after 120 steps ({st})")


@pytest.mark.parametrize("kmax,owned,band", [(1, 64, 0.0), (3, 96, 0.6), (8, 64, 0.0), (16, 256, 1.2)])
def test_tile_shapes_bit_exact(rb, oracle, kmax, owned, band):
    """4,096 spheres (C2), small tiles (many tiles, thin bands: redos and
    restarts happen), several block lengths; 300 steps in 3 calls."""
    sc = scenes.make("c2")
    q, v, st = run_tile(rb, sc, 100, chunks=3, kmax=kmax, owned=owned, band=band)
    assert st["tile_steps"] >= 1, st                   # (a capacity stop finishes on the per-step kernels)
    oracle.set_threads(16)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 300)
    assert_same(q, v, q1, v1, f"c2 kmax={kmax} owned={owned} band={band} ({st})")


def test_tile_dense_pile_bit_exact(rb, oracle):
    """A dense pile (balls_pile geometry, spacing 0.25, lateral speeds 1 m/s,
    spins 3 rad/s) under the default law: many sphere-sphere contacts per
    body, fast bodies; 200 steps."""
    sc = scenes.balls_pile(48, 48, seed=3).with_(restitution=0.8, friction=0.3)
    q, v, st = run_tile(rb, sc, 200, owned=128)
    assert st["tile_runs"] == 1, st
    oracle.set_threads(16)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 200)
    assert_same(q, v, q1, v1, f"dense pile ({st})")


def test_tile_f32_bit_exact_vs_f32_restatement(rb, oracle):
    sc = scenes.make("c3")
    q, v, st = run_tile(rb, sc, 60, dtype="f32")
    assert st["tile_steps"] == 60, st
    oracle.set_threads(16)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 60, dtype="f32")
    assert np.array_equal(q.astype(np.float32), q1.astype(np.float32))
    assert np.array_equal(v.astype(np.float32), v1.astype(np.float32))


def test_tile_then_recorded_step_contacts(rb, oracle):
    """A recorded run: the tile blocks take all but the last step, the last
    runs on the per-step kernel and its contact list equals the oracle's."""
    sc = scenes.make("c3")
    with rb.World(sc) as w:
        w.tile_config(1)
        w.record_contacts(True)
        w.step(40)
        q, v = w.get_state()
        cnt, par, kin, dis = w.contacts()
        st = w.stats()
    assert st["tile_steps"] == 39, st
    oracle.set_threads(16)
    q1, v1, (c1, p1, k1, d1) = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 40, record=True)
    assert_same(q, v, q1, v1, "recorded tile run")
    assert np.array_equal(cnt, c1) and np.array_equal(par, p1) and np.array_equal(kin, k1)
    assert np.array_equal(dis.view(np.uint64), d1.view(np.uint64))


def test_tile_bodies_leaving_the_grid(rb, oracle):
    """Bodies thrown far outside the fitted tile grid land in the edge tiles
    (unbounded outward); still exact."""
    sc = scenes.flat_spheres(96, 96, seed=5)
    qv = sc.qvel0.copy()
    qv[::97, 0:2] = np.random.default_rng(1).normal(0.0, 25.0, (qv[::97].shape[0], 2))
    sc = sc.with_(qvel0=qv)
    q, v, st = run_tile(rb, sc, 150, owned=128)
    oracle.set_threads(16)
    q1, v1 = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 150)
    assert_same(q, v, q1, v1, f"fliers ({st})")


def test_tile_modes_and_counters(rb):
    """Mode 1 takes sphere worlds; mode 0 keeps the per-step kernels; auto
    mode is currently off; box worlds never tile.  The
    counters say which ran."""
    with rb.World(scenes.make("c3")) as w:
        assert w.stats()["tile_on"] == 0          # auto: off
        w.tile_config(1)
        assert w.stats()["tile_on"] == 1
        w.step(16)
        assert w.stats()["tile_steps"] == 16
        w.tile_config(0)
        w.step(16)
        assert w.stats()["tile_steps"] == 16 and w.stats()["tile_on"] == 0
    with rb.World(scenes.make("c5")) as w:
        w.tile_config(1)
        assert w.stats()["tile_on"] == 0          # boxes: per-step kernels
