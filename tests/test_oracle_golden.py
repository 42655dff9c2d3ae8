"""The oracle (C restatement) against vectors produced by the reference's own
functions (tests/golden/make_golden.py).  Bit-exact: the oracle restates the
reference arithmetic in NumPy's operation order."""
import numpy as np
import pytest

from conftest import NBODY_GOLDENS, golden_scene, load_golden


def test_kat_impulse_bit_exact(oracle):
    g = load_golden("kat_impulse")
    out = oracle.kat_impulse(g["inp"])
    assert np.array_equal(out, g["out"]), "a1+a2 KAT mismatch (collision.py:7-48, physics_utils.py:25-49)"


def test_kat_impulse_covers_edge_cases():
    g = load_golden("kat_impulse")
    inp, out = g["inp"], g["out"]
    # separating / exactly-zero normal velocity rows give jn == 0, jt == 0
    assert ((out[:, 0] == 0) & (np.abs(out[:, 1:4]).sum(1) == 0)).sum() >= 2
    # friction cut-off rows around |u_t| = 1e-6
    ut = np.abs(inp[:, 3])
    assert np.any(ut == 1e-6) and np.any(ut == np.nextafter(1e-6, 0)) and np.any(ut == np.nextafter(1e-6, 1))
    assert np.any(inp[:, 1] == 0.0) and np.any(inp[:, 1] == 1.0) and np.any(inp[:, 2] == 0.0)


def test_kat_inertia_bit_exact(oracle):
    g = load_golden("kat_inertia")
    out = oracle.kat_inertia(g["inp"])
    assert np.array_equal(out, g["out"]), "compute_inertia_tensor_world / np.linalg.inv mismatch"


@pytest.mark.parametrize("name", ["traj_single_sphere", "traj_single_cube"])
def test_single_body_trajectory_bit_exact(oracle, name):
    g = load_golden(name)
    sc = golden_scene(g)
    osc = oracle.OracleScene(sc)
    q, v = g["qpos0"], g["qvel0"]
    for t in range(0, 2000, 100):          # 100-step chunks; compare at chunk ends
        q, v = oracle.step(osc, q, v, 100)
        assert np.array_equal(q[0], g["qpos"][t + 100]), f"{name}: qpos differs after step {t + 100}"
        assert np.array_equal(v[0], g["qvel"][t + 100]), f"{name}: qvel differs after step {t + 100}"


def test_single_sphere_reproduces_reference_plot():
    """data/plots/single_sphere/height_vs_time.png: local maxima of
    z at (t, z) = (1.116, 1.478), (2.061, 1.109), (2.871, 0.845), ...
    and x, y drifting to about (0.62, -0.62) by t = 5.2 s."""
    g = load_golden("traj_single_sphere")
    z = g["qpos"][:, 2]
    t = np.arange(len(z)) * 0.009
    peaks = [k for k in range(1, len(z) - 1) if z[k] > z[k - 1] and z[k] >= z[k + 1]]
    got = [(round(t[k], 3), round(z[k], 3)) for k in peaks[:7]]
    want = [(1.116, 1.478), (2.061, 1.109), (2.871, 0.845), (3.555, 0.666), (4.122, 0.541),
            (4.617, 0.451), (5.049, 0.386)]
    for (tg, zg), (tw, zw) in zip(got, want):
        assert abs(tg - tw) <= 0.0095 and abs(zg - zw) <= 0.002, (got, want)
    k = int(round(5.2 / 0.009))
    assert abs(g["qpos"][k, 0] - 0.62) < 0.03 and abs(g["qpos"][k, 1] + 0.62) < 0.03


def test_single_cube_reproduces_reference_plot():
    """data/plots/cube/cube_height_vs_time.png: the cube of
    config 5 (cube_incline.py via timestep_integration, time_integeration.py:13-72;
    dt 0.009, e 0.2, mu 0.6, threshold 1e-4) slides down the 0.7 rad incline,
    its height z read off the reference's committed plot at
    (t, z) = (0.495, 0.207), (0.999, -0.290), (1.494, -1.068), (1.998, -2.155),
    (2.133, -2.497) — the plot ends near -2.47 at about 2.13 s.  Tolerance
    0.03: the plot-reading precision.  This pins the restated plane-box
    contact rule (MuJoCo's mjc_PlaneBox, unavailable offline) that C5 uses."""
    g = load_golden("traj_single_cube")
    dt = float(g["params"][0])
    z = g["qpos"][:, 2]
    for t, want in [(0.495, 0.207), (0.999, -0.290), (1.494, -1.068), (1.998, -2.155), (2.133, -2.497)]:
        k = int(round(t / dt))
        assert abs(z[k] - want) <= 0.03, (t, z[k], want)
    # and the cube keeps sliding (no rest) over the plotted range
    assert np.all(np.diff(z[int(round(0.5 / dt)):int(round(2.13 / dt))]) < 0)


@pytest.mark.parametrize("name", NBODY_GOLDENS)
def test_nbody_trajectory_and_contacts_bit_exact(oracle, name):
    g = load_golden(name)
    sc = golden_scene(g)
    osc = oracle.OracleScene(sc)
    q, v = g["qpos0"], g["qvel0"]
    snaps = list(g["snap_step"])
    si = 1
    for t in range(snaps[-1]):
        q, v, (cnt, par, kin, dis) = oracle.step(osc, q, v, 1, record=True)
        if t < len(g["c_counts"]):
            a, b = g["c_off"][t], g["c_off"][t + 1]
            assert np.array_equal(cnt, g["c_counts"][t]), f"contact counts differ at step {t}"
            assert np.array_equal(par, g["c_partner"][a:b]), f"contact partners differ at step {t}"
            assert np.array_equal(kin, g["c_kind"][a:b]), f"contact kinds differ at step {t}"
            assert np.array_equal(dis, g["c_dist"][a:b]), f"contact dists differ at step {t}"
        if si < len(snaps) and t + 1 == snaps[si]:
            assert np.array_equal(q, g["qpos"][si]), f"qpos differs at step {t + 1}"
            assert np.array_equal(v, g["qvel"][si]), f"qvel differs at step {t + 1}"
            si += 1


def test_goldens_exercise_contacts():
    """The N-body goldens must actually contain plane and sphere-sphere
    contacts (and box corners), or the bit-exact checks above are vacuous."""
    kinds = {n: set(np.unique(load_golden(n)["c_kind"]).tolist()) for n in NBODY_GOLDENS}
    assert 16 in kinds["traj_flat64"] and 0 in kinds["traj_flat64"]
    assert 16 in kinds["traj_flat256"] and 16 in kinds["traj_flat64_raw"]
    assert any(1 <= k <= 8 for k in kinds["traj_cubes16"])


def test_oracle_f32_close_to_f64(oracle):
    """The fp32 restatement (what the f32 kernel must reproduce bit for bit)
    stays near the fp64 trajectory on a non-chaotic scene."""
    g = load_golden("traj_single_sphere")
    sc = golden_scene(g)
    osc = oracle.OracleScene(sc)
    q64, _ = oracle.step(osc, g["qpos0"], g["qvel0"], 300)
    q32, _ = oracle.step(osc, g["qpos0"], g["qvel0"], 300, dtype="f32")
    assert np.abs(q64 - q32).max() < 1e-3


def test_oracle_overlapping_cubes_get_box_contacts(oracle):
    """Two cubes 0.5 apart on the incline (they overlap): box-box contacts
    (rb_oracle_impl.h box_box) in both bodies' lists, the
    same records from either side, normals opposite under ORIENTED."""
    from rbhip import scenes
    sc = scenes.incline_cubes(2, 1, seed=0, spacing=0.5)
    osc = oracle.OracleScene(sc)
    cnt, par, kin, dis, pos, frm = oracle.contacts(osc, sc.qpos0)
    bb = kin >= 32
    assert bb.sum() >= 2 and set(par[bb].tolist()) == {0, 1}
    a, b = (par == 1) & bb, (par == 0) & bb
    assert np.array_equal(dis[a], dis[b]) and np.array_equal(pos[a], pos[b]) and np.array_equal(frm[a], frm[b])
    q, v = oracle.step(osc, sc.qpos0, sc.qvel0, 5)
    assert np.isfinite(q).all()


def test_oracle_thread_count_invariant(oracle):
    """The CPU baseline runs the oracle with OpenMP over bodies: its results
    must not depend on the thread count (bodies are independent within a
    step: Jacobi across bodies, multi_sphere_bounce.py:43-46)."""
    from rbhip import scenes
    sc = scenes.flat_spheres(24, 24, seed=3)
    osc = oracle.OracleScene(sc)
    out = {}
    try:
        for th in (1, 3, 8):
            oracle.set_threads(th)
            out[th] = oracle.step(osc, sc.qpos0, sc.qvel0, 80, record=True)
    finally:
        oracle.set_threads(1)
    q1, v1, c1 = out[1]
    for th in (3, 8):
        q, v, c = out[th]
        assert np.array_equal(q, q1) and np.array_equal(v, v1)
        for a, b in zip(c, c1):
            assert np.array_equal(a, b)


# ---- the two-ball law (ball_collision.py:39-125) ---------------------------

def test_kat_pair_impulse_bit_exact(oracle):
    """compute_collision_impulse (ball_collision.py:53-68) on 1,509 cases,
    including |v_t| around the 1e-8 switch and friction clipped both ways."""
    g = load_golden("kat_pair_impulse")
    assert np.array_equal(oracle.kat_pair_impulse(g["inp"]), g["out"])


@pytest.mark.parametrize("name", ["traj_balls2", "traj_balls2_spin"])
def test_two_ball_trajectory_bit_exact(oracle, name):
    """step_with_custom_collisions (ball_collision.py:73-125), 600 steps, every
    step; the run goes through ground bounces and the ball-ball collision."""
    g = load_golden(name)
    sc = golden_scene(g)
    osc = oracle.OracleScene(sc)
    q, v = sc.qpos0, sc.qvel0
    q1, v1 = oracle.pair_step(osc, sc.qpos0, sc.qvel0, 1, tol=float(g["tol"]))
    assert np.array_equal(q1, g["qpos"][0]) and np.array_equal(v1, g["qvel"][0])
    for t in range(g["qpos"].shape[0]):
        q, v = oracle.pair_step(osc, q, v, 1, tol=float(g["tol"]))
        assert np.array_equal(q, g["qpos"][t]) and np.array_equal(v, g["qvel"][t]), t
    qn, vn = oracle.pair_step(osc, sc.qpos0, sc.qvel0, g["qpos"].shape[0], tol=float(g["tol"]))
    assert np.array_equal(qn, g["qpos"][-1]) and np.array_equal(vn, g["qvel"][-1])
    d = np.linalg.norm(g["qpos"][:, 1, :3] - g["qpos"][:, 0, :3], axis=1)
    assert d.min() < 0.21 and g["qpos"][:, :, 2].min() < 0.1      # both contact kinds happened


def test_ball_law_pile_pairs(oracle):
    """N-ball generalisation: pairs found are exactly those within r_a + r_b
    + tol (brute force on the post-ground positions of the last step)."""
    from rbhip import scenes
    sc = scenes.balls_pile(8, 8, seed=1)
    osc = oracle.OracleScene(sc)
    q, v = oracle.pair_step(osc, sc.qpos0, sc.qvel0, 60)
    q2, v2, (cnt, par) = oracle.pair_step(osc, q, v, 1, record=True)
    assert cnt.sum() > 0 and cnt.sum() % 2 == 0
    # rebuild the post-ground positions and check the pair set
    p = q[:, :3].copy()
    p[:, 2] = np.where(p[:, 2] < 0.1, 0.1, p[:, 2])
    off = np.concatenate([[0], np.cumsum(cnt)])
    for i in range(sc.n):
        want = [j for j in range(sc.n) if j != i and np.linalg.norm(p[max(i, j)] - p[min(i, j)]) < 0.21]
        assert list(par[off[i]:off[i + 1]]) == want
