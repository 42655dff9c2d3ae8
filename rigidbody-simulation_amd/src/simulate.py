"""Headless runner with the reference's simulation names (src/simulate.py),
stepping on the GPU: `python -m src.simulate --sim NAME [--steps N]`.

The reference launches each scene script in a subprocess that opens a GLFW
viewer and steps once per rendered frame (simulate.py:9-37,
mujoco_viewer.py:106-139).  Here a scene runs headless for --steps steps on
one MI355X; positions are sampled every --log-every steps into the
reference's logger classes (src/visualization) and saved under --out
(trajectory .npz, and the reference's plots when matplotlib is present).
MuJoCo stays out of the loop: scenes come from rbhip.scenes or, with
--model, from the reference's MJCF files through rbhip.mjcf.
"""
import argparse
import os
import sys

import numpy as np

# per scene: the parameters the reference scripts pass (sim_overrides.py,
# the step functions' defaults) and the logger they fill
SIMS = {
    # single_sphere_bounce.py:40-41, :65-69 -> collision.py:56 (threshold 0)
    "single_sphere": dict(scene="single_sphere", law="mujoco", e=1.0, mu=0.5, thr=0.0, spin=(2.0, 2.0, 0.0)),
    # cube_incline.py:44, :75-77 -> time_integeration.py:13 (threshold 1e-4)
    "cube_incline": dict(scene="single_cube", law="mujoco", e=0.2, mu=0.6, thr=1e-4),
    # multi_sphere_bounce.py (sim_overrides.py:22-27)
    "multi_sphere": dict(scene="multi_sphere", law="mujoco", e=1.0, mu=0.0, thr=0.0),
    # ball_collision.py:31-34, :73-125 (sim_overrides.py:16-21)
    "ball_collision": dict(scene="ball_collision", law="balls", e=1.0, mu=0.3, thr=0.0, tol=0.01),
}
UNSUPPORTED = {"compare_builtin": "compare_builtin_simulation.py runs MuJoCo's own solver (mj_step); "
                                  "it is the reference's comparison baseline, not this stepper"}


def build_scene(name: str, model_path=None):
    """The scene of a simulation name, with the reference script's initial
    conditions applied (also on top of an MJCF model)."""
    from rbhip import mjcf, scenes
    cfg = SIMS[name]
    base = scenes.make(cfg["scene"])
    if model_path is None:
        return base
    sc = mjcf.load(model_path, restitution=cfg["e"], friction=cfg["mu"], threshold=cfg["thr"])
    if sc.n != base.n:
        raise ValueError(f"{model_path}: {sc.n} free bodies, the {name} scene has {base.n}")
    qvel = np.zeros((sc.n, 6))
    qpos = sc.qpos0.copy()
    if "spin" in cfg:
        qvel[0, 3:6] = cfg["spin"]
    if name == "ball_collision":                 # ball_collision.py:31-34
        qpos[:, 0:3], qvel[:, 0:3] = base.qpos0[:, 0:3], base.qvel0[:, 0:3]
    return sc.with_(qpos0=qpos, qvel0=qvel)


def run(name: str, steps: int, log_every: int = 1, model_path=None, dtype: str = "f64", out=None):
    """Step the scene on the GPU; returns (final qpos, final qvel, logger)."""
    import rbhip
    from rbhip.sampling import run_sampled
    from src.visualization.data_logger import DataLogger
    from src.visualization.multi_sphere_logger import MultiSphereLogger
    cfg = SIMS[name]
    sc = build_scene(name, model_path)
    names = sc.names or [f"body{k}" for k in range(sc.n)]
    logger = DataLogger() if sc.n == 1 else MultiSphereLogger(names)

    def sample(step, t, q, v):
        if sc.n == 1:
            logger.record(t, q[0, 2], q[0, 0], q[0, 1])
        else:
            logger.record_all(t, q)

    with rbhip.World(sc, dtype=dtype, law=cfg["law"], tol=cfg.get("tol", 0.01)) as w:
        run_sampled(w, steps, log_every, sample, restitution=cfg["e"], friction=cfg["mu"], threshold=cfg["thr"])
        q, v = w.get_state()
    if out:
        os.makedirs(out, exist_ok=True)
        logger.save_npz(os.path.join(out, f"{name}_trajectory.npz"))
        try:
            import matplotlib  # noqa: F401
        except ImportError:
            pass
        else:
            if sc.n == 1:
                logger.save_plot(os.path.join(out, f"{name}_height_vs_time.png"))
                logger.save_trajectory_plot_3d(os.path.join(out, f"{name}_trajectory_3d.png"))
            else:
                logger.save_all_plots(os.path.join(out, name))
    return q, v, logger


def main(argv=None):
    ap = argparse.ArgumentParser(description="Headless GPU runner of the reference's simulations")
    ap.add_argument("--sim", required=True,
                    help="Simulation to run. Available: " + ", ".join(list(SIMS) + list(UNSUPPORTED)))
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--log-every", type=int, default=1, help="sample positions every K steps")
    ap.add_argument("--model", default=None, help="MJCF file to load instead of the built-in scene")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--out", default=None, help="directory for the trajectory (.npz) and plots")
    args = ap.parse_args(argv)
    if args.sim in UNSUPPORTED:
        print(f"{args.sim}: not available headless: {UNSUPPORTED[args.sim]}", file=sys.stderr)
        return 2
    if args.sim not in SIMS:
        print(f"Unknown simulation name: {args.sim!r}. Available: {', '.join(SIMS)}", file=sys.stderr)
        return 1
    q, v, _ = run(args.sim, args.steps, args.log_every, args.model, args.dtype, args.out)
    for k, row in enumerate(q):
        print(f"body {k}: x = {row[0]:+.6f} {row[1]:+.6f} {row[2]:+.6f}  |v| = {np.linalg.norm(v[k, :3]):.6f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
