"""The box-involved narrowphase of the oracle on
analytic cases, on CPU.  MuJoCo's mjc_SphereBox / mjc_BoxBox are not
available offline, so the oracle's sphere_box / box_box are this project's
definition (rb_oracle_impl.h "box pairs"); these cases pin their geometry —
depth, contact points, normal direction geom1 -> geom2 — not MuJoCo itself
(parity against MuJoCo is unpinned).  The HIP path is checked against the
same oracle bit for bit in tests/test_gpu_boxes.py."""
import numpy as np
import pytest

I = [1.0, 0.0, 0.0, 0.0]
SPHERE, BOX = 0, 1


def row(k1, c1, q1, s1, k2, c2, q2, s2):
    return np.array([k1, k2, *c1, *q1, *s1, *c2, *q2, *s2], float)


def contacts(out):
    n = int(out[0])
    return [(out[1 + 8 * t], out[2 + 8 * t:5 + 8 * t], out[5 + 8 * t:8 + 8 * t], int(out[8 + 8 * t])) for t in range(n)]


def test_face_stack_four_points(oracle):
    out = oracle.kat_narrow(row(BOX, [0, 0, 0], I, [.4, .4, .4], BOX, [0, 0, 0.79], I, [.4, .4, .4])[None])[0]
    cs = contacts(out)
    assert len(cs) == 4
    for t, (d, p, f, k) in enumerate(cs):
        assert d == pytest.approx(-0.01) and np.allclose(f, [0, 0, 1]) and k == 32 + t
        assert p[2] == pytest.approx(0.395) and np.allclose(np.abs(p[:2]), 0.4)


def test_offset_face_clip_inside_overlap():
    """B shifted by (0.5, 0.3): the clipped points are the corners of the
    overlap rectangle [0.1, 0.4] x [-0.1, 0.4]."""
    from oracle import oracle
    out = oracle.kat_narrow(row(BOX, [0, 0, 0], I, [.4, .4, .4], BOX, [0.5, 0.3, 0.78], I, [.4, .4, .4])[None])[0]
    pts = sorted(tuple(np.round(p[:2], 12)) for _, p, _, _ in contacts(out))
    assert pts == sorted([(0.1, -0.1), (0.4, -0.1), (0.4, 0.4), (0.1, 0.4)])


def test_sphere_on_box_top(oracle):
    out = oracle.kat_narrow(row(SPHERE, [0, 0, 0.45], I, [.1, 0, 0], BOX, [0, 0, 0], I, [.4, .4, .4])[None])[0]
    (d, p, f, k), = contacts(out)
    assert d == pytest.approx(-0.05) and np.allclose(p, [0, 0, 0.375]) and np.allclose(f, [0, 0, -1]) and k == 17


def test_sphere_centre_inside_box(oracle):
    out = oracle.kat_narrow(row(SPHERE, [0.1, 0, 0.3], I, [.1, 0, 0], BOX, [0, 0, 0], I, [.4, .4, .4])[None])[0]
    (d, p, f, k), = contacts(out)
    assert d == pytest.approx(-0.2) and np.allclose(f, [0, 0, -1]) and np.allclose(p, [0.1, 0, 0.3])


def test_box_then_sphere_keeps_sphere_as_geom1(oracle):
    """Body order box (lower id), sphere: MuJoCo dispatches sphere-box with
    the sphere as geom1, so the frame still points sphere -> box."""
    out = oracle.kat_narrow(row(BOX, [0, 0, 0], I, [.4, .4, .4], SPHERE, [0, 0, 0.45], I, [.1, 0, 0])[None])[0]
    (d, p, f, k), = contacts(out)
    assert np.allclose(f, [0, 0, -1]) and d == pytest.approx(-0.05)


def test_edge_edge(oracle):
    a = np.pi / 4
    qx = [np.cos(a / 2), np.sin(a / 2), 0, 0]
    qy = [np.cos(a / 2), 0, np.sin(a / 2), 0]
    zb = 0.4 * np.sqrt(2) * 2 - 0.02
    out = oracle.kat_narrow(row(BOX, [0, 0, 0], qx, [.4, .4, .4], BOX, [0.05, 0.03, zb], qy, [.4, .4, .4])[None])[0]
    (d, p, f, k), = contacts(out)
    assert k == 40 and d == pytest.approx(-0.02) and np.allclose(f, [0, 0, 1])
    assert np.allclose(p, [0.05, 0.0, 0.4 * np.sqrt(2) - 0.01])


def test_separated_and_random_pairs_are_finite(oracle):
    rng = np.random.default_rng(0)
    rows = []
    for _ in range(3000):
        k1, k2 = rng.integers(0, 2, 2)
        q1, q2 = rng.normal(size=4), rng.normal(size=4)
        s1 = [.1, 0, 0] if k1 == 0 else list(rng.uniform(.1, .5, 3))
        s2 = [.1, 0, 0] if k2 == 0 else list(rng.uniform(.1, .5, 3))
        rows.append(row(k1, [0, 0, 0], q1 / np.linalg.norm(q1), s1, k2, rng.uniform(-.8, .8, 3),
                        q2 / np.linalg.norm(q2), s2))
    out = oracle.kat_narrow(np.array(rows))
    assert np.isfinite(out).all()
    n = out[:, 0].astype(int)
    assert n.max() <= 4 and (n > 0).sum() > 300
    d = np.concatenate([out[r, 1:1 + 8 * n[r]:8] for r in range(len(rows))])
    assert (d <= 0).all()
    kinds = {int(k) for r in range(len(rows)) for k in out[r, 8:8 + 8 * n[r]:8]}
    assert {16, 17, 32, 33, 34, 35, 40} <= kinds


def test_box_pile_steps_all_contact_kinds(oracle):
    """The oracle steps the box pile (cube.xml-sized boxes stacked in tilted
    columns, sphere caps) through face, edge and sphere-box contacts and
    stays bounded."""
    from rbhip import scenes
    sc = scenes.box_pile(4, 4, 3, seed=1)
    osc = oracle.OracleScene(sc, max_partners=32)
    q, v = sc.qpos0, sc.qvel0
    seen = set()
    for _ in range(6):
        q, v = oracle.step(osc, q, v, 49)
        q, v, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
        seen |= set(kin.tolist())
    assert {17, 32, 40} <= seen and np.isfinite(q).all() and np.abs(v).max() < 100
