"""Mirror of src/simulation/multi_sphere_bounce.py's N-body step.

Unlike the reference script this module has no import-time side effects
(the reference opens a GLFW window and runs its viewer at import,
multi_sphere_bounce.py:104-122); `main()` runs the scene headless.

Parity decisions: D1 fixed — body k (0-based among free
bodies) lives at qpos[7k:7k+7], qvel[6k:6k+6]; D2 fixed — contacts are
associated with bodies by index; D8 — normal_convention "oriented"
(default) or "raw".
"""
import numpy as np

from rbhip import adapter, scenes

# sim_overrides.py:22-27 (multi_sphere_bounce)
FRICTION_COEFFICIENT = 0.0
RESTITUTION = 1.0
TIMESTEP = 0.01
friction_coefficient = FRICTION_COEFFICIENT
restitution_coefficient = RESTITUTION
timestep = TIMESTEP
ball_names = ["ball1", "ball2", "ball3", "ball4"]


def custom_step_multi_sphere(model, data, dt=timestep, restitution=restitution_coefficient,
                             friction_coeff=None, contact_threshold=0.0, logger=None,
                             normal_convention="oriented"):
    """multi_sphere_bounce.py:42-92 — one contact pass for the whole scene,
    then every body: gravity, impulses over its contacts (dist < 0), and
    semi-implicit integration.  Returns None; optional logger.record(name,
    t, pos) per body as the reference does (:90)."""
    mu = friction_coefficient if friction_coeff is None else friction_coeff
    adapter.step_model(model, data, 1, dt, restitution, mu, contact_threshold, normal_convention)
    if logger is not None:
        names = getattr(model, "names", None)
        q = np.asarray(data.qpos).reshape(-1, 7)
        for k in range(q.shape[0]):
            name = names[adapter.SceneModel.FIRST + k] if names else f"body{k}"
            logger.record(name, getattr(data, "time", 0.0), q[k, 0:3].copy())
    return None


def load_model():
    """The models/multi_sphere.xml scene as (model, data)."""
    return adapter.load_scene_model(scenes.multi_sphere4())


def main(steps: int = 1000):
    model, data = load_model()
    for _ in range(steps):
        custom_step_multi_sphere(model, data)
    return np.asarray(data.qpos).reshape(-1, 7)


if __name__ == "__main__":
    print(main())
