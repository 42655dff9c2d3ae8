"""Box-involved contacts on the HIP path, through the
C-ABI, against the oracle's restatement (rb_oracle_impl.h "box pairs"; this
project's definition of MuJoCo's sphere-box / box-box primitives — parity
against MuJoCo itself is unpinned).  Bar: fp64 bit-exact (contact counts,
partners, kinds, distances and state), fp32 bit-exact against the fp32
restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


def _same(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint64),
                                                 np.ascontiguousarray(b).view(np.uint64))


def _random_pairs(n, seed=0):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        k1, k2 = rng.integers(0, 2, 2)
        q1, q2 = rng.normal(size=4), rng.normal(size=4)
        s1 = [.1, 0, 0] if k1 == 0 else list(rng.uniform(.1, .5, 3))
        s2 = [.1, 0, 0] if k2 == 0 else list(rng.uniform(.1, .5, 3))
        c2 = rng.uniform(-.8, .8, 3)
        if rng.random() < 0.1:
            c2 = rng.uniform(-.05, .05, 3)             # deep: sphere centre inside the box
        rows.append([k1, k2, 0, 0, 0, *(q1 / np.linalg.norm(q1)), *s1, *c2, *(q2 / np.linalg.norm(q2)), *s2])
    # axis-aligned stacks: parallel edges (skipped axes) and face-face clipping
    for dz in (0.79, 0.7, 0.5):
        for dx in (0.0, 0.3, 0.6):
            rows.append([1, 1, 0, 0, 0, 1, 0, 0, 0, .4, .4, .4, dx, 0.1, dz, 1, 0, 0, 0, .4, .4, .4])
    return np.array(rows, float)


def test_kat_narrow_device_bit_exact(rb, oracle):
    inp = _random_pairs(6000)
    ref = oracle.kat_narrow(inp)
    out = rb.kat_narrow(inp)
    bad = np.nonzero((out.view(np.uint64) != ref.view(np.uint64)).any(1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}: {out[bad[:1]]} vs {ref[bad[:1]]}"
    n = ref[:, 0].astype(int)
    kinds = {int(k) for r in range(len(inp)) for k in ref[r, 8:8 + 8 * n[r]:8]}
    assert {16, 17, 32, 33, 34, 35, 40} <= kinds


def test_kat_narrow_f32_matches_f32_restatement(rb, oracle):
    inp = _random_pairs(2000, seed=1)
    assert np.array_equal(rb.kat_narrow(inp, dtype="f32"), oracle.kat_narrow(inp, dtype="f32"))


@pytest.mark.parametrize("form,env", [("coop", {}), ("wide", {"RBHIP_COOP_MAX_BODIES": "0"}),
                                      ("wide_plain", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_HELP": "0"}),
                                      ("one", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_MAX_BODIES": "0"})])
def test_box_pile_bit_exact(rb, oracle, monkeypatch, form, env):
    """Tilted cube columns with sphere caps (rbhip.scenes.box_pile) landing,
    stacking, leaning and toppling: every step of two recorded windows
    (contacts and state) and the state every 100 steps bit-exact with the
    oracle over 600 steps, with face-clip, edge-edge and sphere-box contacts
    all present — through the cooperative, wide and one-lane sphere forms
    (each followed by the box kernel; "one" is what every box world above
    65,536 bodies runs)."""
    from rbhip import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = scenes.box_pile(6, 6, 3, seed=0)
    osc = oracle.OracleScene(sc, max_partners=32)
    q, v = sc.qpos0, sc.qvel0
    seen = set()
    with rb.World(sc, max_partners=32) as w:
        for t in range(0, 600, 100):
            if t in (100, 400):
                w.record_contacts(True)
                for s in range(t + 1, t + 21):
                    q, v, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
                    w.step(1)
                    gc, gp, gk, gd = w.contacts()
                    assert np.array_equal(gc, cnt), f"contact counts differ at step {s}"
                    assert np.array_equal(gp, par) and np.array_equal(gk, kin), f"partners/kinds differ at step {s}"
                    assert _same(gd, dis), f"contact distances differ at step {s}"
                    seen |= set(kin.tolist())
                w.record_contacts(False)
                q, v = oracle.step(osc, q, v, 80)
                w.step(80)
            else:
                q, v = oracle.step(osc, q, v, 100)
                w.step(100)
            gq, gv = w.get_state()
            assert _same(gq, q) and _same(gv, v), f"state differs after step {t + 100}"
        st = w.stats()
    assert {17, 32, 40} <= seen and (np.array(sorted(seen)) >= 1).any()
    # chunks replayed without the box kernel were rolled back (bodies deferred)
    assert st["box_opt_chunks"] >= 1 and st["box_rollbacks"] >= 1, st


def test_box_pile_f32_bit_exact(rb, oracle):
    from rbhip import scenes
    sc = scenes.box_pile(4, 4, 3, seed=2)
    q0, v0 = oracle.step(oracle.OracleScene(sc, max_partners=32), sc.qpos0, sc.qvel0, 300, dtype="f32")
    with rb.World(sc, dtype="f32", max_partners=32) as w:
        w.step(300)
        q, v = w.get_state()
    assert np.array_equal(q, q0) and np.array_equal(v, v0)


def _approaching_boxes():
    """Two spinning cubes and a sphere thrown at each other in the air: for
    the first 7 steps no box-involved pair is within bounding range (the
    sphere step kernel steps the cubes), then the cubes meet face to face in
    the very step their bounding spheres first overlap (the box kernel takes
    them over and reads both step-start orientations)."""
    from rbhip import scenes
    h = 0.4
    kind = np.array([1, 1, 0], np.int32)
    mass = np.array([scenes.M_CUBE_H04, scenes.M_CUBE_H04, scenes.M_SPHERE_R02])
    inertia = np.array([[scenes.I_CUBE_H04] * 3, [scenes.I_CUBE_H04] * 3, [scenes.I_SPHERE_R02] * 3])
    size = np.array([[h, h, h], [h, h, h], [0.2, 0, 0]])
    qpos = np.array([[-2.5, 0.0, 3.0, 1, 0, 0, 0], [2.5, 0.1, 3.0, 1, 0, 0, 0], [0.1, 2.2, 3.1, 1, 0, 0, 0]], float)
    qvel = np.array([[30.0, 0, 0, 1.0, 2.0, 0.5], [-30.0, 0, 0, -0.5, 1.0, 2.0], [0, -3.5, 0, 0, 0, 0]], float)
    return scenes.Scene("approaching_boxes", kind, mass, inertia, size, np.array([[0.0, 0, 1, 0, 0, 0]]),
                        qpos, qvel, dt=0.01, restitution=0.5, friction=0.4, threshold=0.0)


@pytest.mark.parametrize("form,env", [("coop", {}), ("wide", {"RBHIP_COOP_MAX_BODIES": "0"}),
                                      ("wide_plain", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_HELP": "0"}),
                                      ("one", {"RBHIP_COOP_MAX_BODIES": "0", "RBHIP_WIDE_MAX_BODIES": "0"})])
def test_boxes_entering_range_bit_exact(rb, oracle, monkeypatch, form, env):
    """Boxes stepped by the sphere kernel (no box partner in range) must
    still publish their orientation for the step a box pair comes into
    range: every step's contacts and state bit-exact with the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = _approaching_boxes()
    osc = oracle.OracleScene(sc, max_partners=32)
    q, v = sc.qpos0, sc.qvel0
    kinds = set()
    with rb.World(sc, max_partners=32) as w:
        w.record_contacts(True)
        for s in range(1, 151):
            q, v, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
            w.step(1)
            gc, gp, gk, gd = w.contacts()
            assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin), \
                f"contacts differ at step {s}"
            gq, gv = w.get_state()
            assert _same(gq, q) and _same(gv, v), f"state differs at step {s}"
            kinds |= set(kin.tolist())
    assert {32, 40} <= kinds, kinds


@pytest.mark.parametrize("optimistic", ["1", "0"])
def test_boxes_entering_range_chunked(rb, oracle, monkeypatch, optimistic):
    """The same scene in one 150-step call: replayed without the box kernel
    (rb_world::box_opt), the chunk defers the cubes when they meet, is rolled
    back to its start and replayed with the box kernel; bit-exact either way."""
    monkeypatch.setenv("RBHIP_BOX_OPTIMISTIC", optimistic)
    sc = _approaching_boxes()
    q, v = oracle.step(oracle.OracleScene(sc, max_partners=32), sc.qpos0, sc.qvel0, 150)
    with rb.World(sc, max_partners=32) as w:
        w.step(150)
        gq, gv = w.get_state()
        st = w.stats()
    assert _same(gq, q) and _same(gv, v)
    if optimistic == "1":
        assert st["box_opt_chunks"] == 1 and st["box_rollbacks"] == 1, st
    else:
        assert st["box_opt_chunks"] == 0, st
