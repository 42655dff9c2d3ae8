"""The reference call surface (src.physics.*, src.simulation.multi_sphere_bounce)
backed by the GPU, against the reference's own outputs (goldens)."""
import numpy as np
import pytest

from conftest import golden_scene, load_golden

pytestmark = pytest.mark.gpu


def test_compute_collision_impulse_friction_matches_reference():
    from src.physics.collision import compute_collision_impulse_friction
    g = load_golden("kat_impulse")
    inp, out = g["inp"], g["out"]
    for k in list(range(0, len(inp), 97)) + list(range(len(inp) - 10, len(inp))):
        r = inp[k]
        jn, jt = compute_collision_impulse_friction(r[0], r[15:24].reshape(3, 3), r[3:6], r[6:9], r[9:12],
                                                    r[12:15], r[1], r[2])
        assert isinstance(jn, float) and jt.shape == (3,)
        assert jn == out[k, 0] and np.array_equal(jt, out[k, 1:4])
    # batched form: one launch for every row
    jn, jt = compute_collision_impulse_friction(inp[:, 0], inp[:, 15:24], inp[:, 3:6], inp[:, 6:9],
                                                inp[:, 9:12], inp[:, 12:15], 0.0, 0.0)
    assert jn.shape == (len(inp),)


def test_apply_impulse_friction_matches_reference():
    from src.physics.physics_utils import apply_impulse_friction
    g = load_golden("kat_impulse")
    inp, out = g["inp"], g["out"]
    v, w = apply_impulse_friction(inp[:, 3:6], inp[:, 6:9], inp[:, 0], inp[:, 15:24], inp[:, 9:12],
                                  inp[:, 12:15], out[:, 0], out[:, 1:4])
    assert np.array_equal(v, out[:, 4:7]) and np.array_equal(w, out[:, 7:10])
    v1, w1 = apply_impulse_friction(inp[5, 3:6], inp[5, 6:9], inp[5, 0], inp[5, 15:24].reshape(3, 3),
                                    inp[5, 9:12], inp[5, 12:15], out[5, 0], out[5, 1:4])
    assert v1.shape == (3,) and np.array_equal(v1, out[5, 4:7]) and np.array_equal(w1, out[5, 7:10])


def test_compute_inertia_tensor_world_matches_reference():
    from src.physics.collision import compute_inertia_tensor_world
    g = load_golden("kat_inertia")
    for k in range(0, len(g["inp"]), 50):
        Iw = compute_inertia_tensor_world(g["inp"][k, 0:3], g["inp"][k, 3:7])
        assert np.array_equal(Iw.reshape(9), g["out"][k, 0:9])


def _model_data(name):
    from rbhip import adapter
    g = load_golden(name)
    sc = golden_scene(g)
    if name == "traj_single_sphere":
        sc = sc.with_(names=["ball"])
    elif name == "traj_single_cube":
        sc = sc.with_(names=["cube"])
    m, d = adapter.load_scene_model(sc)
    return g, sc, m, d


def test_single_sphere_step_function_drop_in():
    """single_sphere_bounce.py:65-69 drives the step with obj "sphere" (body
    is "ball": SURVEY D4 — the last body is used, with a warning)."""
    from src.physics.collision import custom_step_with_impulse_collision_friction
    g, sc, model, data = _model_data("traj_single_sphere")
    with pytest.warns(UserWarning, match="D4"):
        pos = custom_step_with_impulse_collision_friction(model, "sphere", data, dt=0.009, restitution=1.0,
                                                          friction_coeff=0.5)
    assert pos.shape == (3,)
    for t in range(1, 300):
        custom_step_with_impulse_collision_friction(model, "ball", data, dt=0.009, restitution=1.0,
                                                    friction_coeff=0.5)
    assert np.array_equal(data.qpos, g["qpos"][300]) and np.array_equal(data.qvel, g["qvel"][300])


def test_cube_timestep_integration_drop_in():
    from src.physics.time_integeration import timestep_integration
    g, sc, model, data = _model_data("traj_single_cube")
    for _ in range(300):
        timestep_integration(model, "cube", data, dt=0.009, restitution=0.2, friction_coeff=0.6)
    assert np.array_equal(data.qpos, g["qpos"][300]) and np.array_equal(data.qvel, g["qvel"][300])


def test_multi_sphere_step_drop_in():
    from src.simulation.multi_sphere_bounce import custom_step_multi_sphere

    class Logger:
        def __init__(self):
            self.n = 0

        def record(self, name, t, pos):
            self.n += 1

    g, sc, model, data = _model_data("traj_multi4")
    log = Logger()
    for _ in range(100):
        custom_step_multi_sphere(model, data, dt=0.01, restitution=1.0, logger=log)
    k = list(g["snap_step"]).index(100)
    assert np.array_equal(np.asarray(data.qpos).reshape(-1, 7), g["qpos"][k])
    assert log.n == 400


# ---- the headless runner (src/simulate.py) ---------------------------------
@pytest.mark.parametrize("sim,golden,steps", [("single_sphere", "traj_single_sphere", 300),
                                              ("cube_incline", "traj_single_cube", 300),
                                              ("ball_collision", "traj_balls2", 300)])
def test_simulate_runs_match_reference(sim, golden, steps, tmp_path):
    from src import simulate
    g = load_golden(golden)
    q, v, logger = simulate.run(sim, steps, log_every=10, out=str(tmp_path))
    # single-body goldens hold the initial state at row 0; the two-ball one starts after step 1
    gq, gv = (g["qpos"][steps][None], g["qvel"][steps][None]) if g["qpos"].ndim == 2 else \
        (g["qpos"][steps - 1], g["qvel"][steps - 1])
    assert np.array_equal(q, gq) and np.array_equal(v, gv)
    traj = np.load(tmp_path / f"{sim}_trajectory.npz")
    assert len(traj.files) >= 1
    if sim != "ball_collision":
        t = traj["trajectory"]
        assert t.shape == (steps // 10, 4) and np.array_equal(t[-1, 1:], gq[0, :3])


def test_simulate_multi_sphere_vs_oracle(oracle):
    from src import simulate
    from rbhip import scenes
    sc = scenes.multi_sphere4()
    qo, vo = oracle.step(oracle.OracleScene(sc), sc.qpos0, sc.qvel0, 250)
    q, v, logger = simulate.run("multi_sphere", 250, log_every=50)
    assert np.array_equal(q, qo) and np.array_equal(v, vo)
    assert len(logger.loggers["ball1"].times) == 5


@pytest.mark.parametrize("entry", ["timestep_integration", "custom_step_with_impulse_collision_friction"])
def test_single_body_entry_on_multi_body_scene(oracle, entry):
    """time_integeration.py:13-72 / collision.py:56-102 called for one named
    body of a scene with several (contacts filtered by body):
    that body alone steps — gravity, its plane and partner contacts against
    the others' step-start positions, integration — and the others stay
    put.  Checked bit for bit against the oracle stepping the same body
    (the oracle steps all, then keeps only that body's row)."""
    from rbhip import adapter
    import src.physics.collision as col
    import src.physics.time_integeration as ti
    g = load_golden("traj_flat64")
    sc = golden_scene(g)
    names = [f"ball{k}" for k in range(sc.n)]
    sc = sc.with_(names=names)
    model, data = adapter.load_scene_model(sc)
    fn = getattr(ti if entry == "timestep_integration" else col, entry)
    osc = oracle.OracleScene(sc)
    q, v = sc.qpos0.copy(), sc.qvel0.copy()
    rng = np.random.default_rng(3)
    thr = 1e-4 if entry == "timestep_integration" else 0.0
    for t in range(160):
        k = int(rng.integers(sc.n)) if t % 4 else 5      # body 5 often: it lands and touches neighbours
        pos = fn(model, names[k], data, dt=sc.dt, restitution=sc.restitution, friction_coeff=sc.friction,
                 contact_threshold=thr)
        q1, v1 = oracle.step(osc, q, v, 1, dt=sc.dt, restitution=sc.restitution, friction=sc.friction, threshold=thr)
        q[k], v[k] = q1[k], v1[k]
        assert np.array_equal(pos, q[k, 0:3])
        assert np.array_equal(np.asarray(data.qpos).reshape(-1, 7), q), f"qpos differs after call {t}"
        assert np.array_equal(np.asarray(data.qvel).reshape(-1, 6), v), f"qvel differs after call {t}"
