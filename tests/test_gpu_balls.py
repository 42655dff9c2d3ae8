"""The two-ball law (ball_collision.py:39-125) on the GPU (RB_LAW_BALLS),
through the C-ABI: against the goldens produced by the reference's own
functions (two balls) and against the oracle's N-ball generalisation.
Bar: fp64 bit-exact; fp32 bit-exact against the fp32 restatement."""
import numpy as np
import pytest

from conftest import golden_scene, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


def test_kat_pair_impulse_device_bit_exact(rb, oracle):
    g = load_golden("kat_pair_impulse")
    out = rb.kat_pair_impulse(g["inp"])
    bad = np.nonzero((out != g["out"]).any(1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}"
    assert np.array_equal(rb.kat_pair_impulse(g["inp"], dtype="f32"), oracle.kat_pair_impulse(g["inp"], dtype="f32"))


@pytest.mark.parametrize("name", ["traj_balls2", "traj_balls2_spin"])
def test_two_balls_vs_reference_every_step(rb, name):
    g = load_golden(name)
    tol = float(g["tol"])
    with rb.World(golden_scene(g), law="balls", tol=tol) as w:
        for t in range(g["qpos"].shape[0]):
            w.step(1)
            q, v = w.get_state()
            assert np.array_equal(q, g["qpos"][t]) and np.array_equal(v, g["qvel"][t]), f"step {t}"


@pytest.mark.parametrize("name", ["traj_balls2", "traj_balls2_spin"])
def test_two_balls_graph_replay(rb, name):
    """The same run as graph-replayed chunks (the post-ground snapshot carried
    from step to step on the device)."""
    g = load_golden(name)
    with rb.World(golden_scene(g), law="balls", tol=float(g["tol"])) as w:
        for k in (1, 99, 200, 300):
            w.step(k)
        q, v = w.get_state()
    assert np.array_equal(q, g["qpos"][-1]) and np.array_equal(v, g["qvel"][-1])


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_ball_pile_vs_oracle(rb, oracle, dtype):
    """N-ball generalisation (Jacobi over pairs) on 256 balls: state and the
    last step's pair lists bit-exact against the oracle."""
    sc = rb.scenes.balls_pile(16, 16, seed=2)
    osc = oracle.OracleScene(sc)
    qo, vo = oracle.pair_step(osc, sc.qpos0, sc.qvel0, 80, dtype=dtype)
    qo2, vo2, (cnt, par) = oracle.pair_step(osc, qo, vo, 1, dtype=dtype, record=True)
    assert cnt.sum() > 10
    with rb.World(sc, dtype=dtype, law="balls", tol=0.01) as w:
        w.step(80)
        q, v = w.get_state()
        assert np.array_equal(q, qo) and np.array_equal(v, vo)
        w.record_contacts(True)
        w.step(1)
        c = w.contacts()
        q, v = w.get_state()
    assert np.array_equal(q, qo2) and np.array_equal(v, vo2)
    assert np.array_equal(c[0], cnt) and np.array_equal(c[1], par)


def test_law_switch_round_trip(rb, oracle):
    """mujoco -> balls -> mujoco on one world continues each law's run."""
    sc = rb.scenes.balls_pile(8, 8, seed=3)
    osc = oracle.OracleScene(sc)
    q1, v1 = oracle.step(osc, sc.qpos0, sc.qvel0, 20)
    q2, v2 = oracle.pair_step(osc, q1, v1, 20)
    q3, v3 = oracle.step(osc, q2, v2, 20)
    with rb.World(sc) as w:
        w.step(20)
        w.set_contact_law("balls", 0.01)
        w.step(20)
        q, v = w.get_state()
        assert np.array_equal(q, q2) and np.array_equal(v, v2)
        w.set_contact_law("mujoco")
        w.step(20)
        q, v = w.get_state()
    assert np.array_equal(q, q3) and np.array_equal(v, v3)


def test_ball_law_parameters_change_reprimes(rb, oracle):
    """The post-ground snapshot depends on dt, e, mu: changing them between
    calls re-runs the ground phase from the true state."""
    sc = rb.scenes.balls_pile(6, 6, seed=4)
    osc = oracle.OracleScene(sc)
    q1, v1 = oracle.pair_step(osc, sc.qpos0, sc.qvel0, 30)
    q2, v2 = oracle.pair_step(osc, q1, v1, 30, dt=0.005, restitution=0.5, friction=0.7)
    with rb.World(sc, law="balls") as w:
        w.step(30)
        w.step(30, dt=0.005, restitution=0.5, friction=0.7)
        q, v = w.get_state()
    assert np.array_equal(q, q2) and np.array_equal(v, v2)


def test_ball_law_rejects_unsupported_scenes(rb):
    for sc in (rb.scenes.single_cube(), rb.scenes.incline_spheres(2, 2)):
        with pytest.raises(rb.RbError) as ei:
            rb.World(sc, law="balls")
        assert ei.value.code == -95


def test_shim_step_and_impulse(rb):
    from src.simulation import ball_collision as bc
    g = load_golden("traj_balls2_spin")
    model, data = bc.load_model()
    sc = golden_scene(g)
    data.qpos[:] = sc.qpos0.reshape(-1)
    data.qvel[:] = sc.qvel0.reshape(-1)
    for t in range(150):
        p1, p2 = bc.step_with_custom_collisions(model, data)
        assert np.array_equal(np.asarray(data.qpos).reshape(-1, 7), g["qpos"][t])
    assert np.array_equal(p2, g["qpos"][149][1, :3])
    k = load_golden("kat_pair_impulse")
    r = k["inp"][:64]
    out = bc.compute_collision_impulse(r[:, 0], r[:, 15:24].reshape(-1, 3, 3), r[:, 3:6], r[:, 6:9], r[:, 9:12],
                                       r[:, 12:15], r[0, 1], r[0, 2])
    same = (r[:, 1] == r[0, 1]) & (r[:, 2] == r[0, 2])
    assert np.array_equal(out[same], k["out"][:64][same])
