"""Mirror of src/simulation/ball_collision.py's contact law, evaluated on the
GPU (librbhip.so, RB_LAW_BALLS).

Unlike the reference script this module has no import-time side effects
(the reference opens a GLFW window and runs its viewer at import,
ball_collision.py:157-189); `main()` runs the scene headless.
"""
import numpy as np

from rbhip import adapter, kat_pair_impulse, scenes

# sim_overrides.py:16-21 (ball_collision); ball_collision.py:23, :102
FRICTION_COEFFICIENT = 0.3
RESTITUTION = 1.0
TIMESTEP = 0.01
friction_coefficient = FRICTION_COEFFICIENT
restitution = RESTITUTION
timestep = TIMESTEP
ball_radius = 0.1
TOL = 0.01


def compute_inverse_inertia(mass, radius):
    """ball_collision.py:39-41 — eye(3) / ((2/5) m r^2) (a scene constant,
    built on the host once)."""
    inertia_val = (2.0 / 5.0) * mass * radius ** 2
    return np.eye(3) / inertia_val


def compute_collision_impulse(mass, I_inv, v_lin, v_ang, r, n, restitution, mu):
    """ball_collision.py:53-68 — the contact impulse jn*n + jt*t_dir (full
    effective mass, friction clipped to mu |jn|), on the GPU.  Batched if the
    vectors carry a leading dimension."""
    v = np.asarray(v_lin, np.float64)
    single = v.ndim == 1
    v = v.reshape(-1, 3)
    B = v.shape[0]
    row = np.zeros((B, 27))
    row[:, 0] = np.broadcast_to(np.asarray(mass, np.float64), (B,))
    row[:, 1] = restitution
    row[:, 2] = mu
    row[:, 3:6] = v
    row[:, 6:9] = np.broadcast_to(np.asarray(v_ang, np.float64).reshape(-1, 3), (B, 3))
    row[:, 9:12] = np.broadcast_to(np.asarray(r, np.float64).reshape(-1, 3), (B, 3))
    row[:, 12:15] = np.broadcast_to(np.asarray(n, np.float64).reshape(-1, 3), (B, 3))
    row[:, 15:24] = np.broadcast_to(np.asarray(I_inv, np.float64).reshape(-1, 9), (B, 9))
    out = kat_pair_impulse(row)
    return out[0].copy() if single else out


def step_with_custom_collisions(model, data, dt=timestep, restitution_coeff=None, friction=None, tol=TOL):
    """ball_collision.py:73-125 — one step of the two-ball law for every ball
    of the scene (gravity, ground contact, ball-ball contacts, x += v dt).
    Mutates data.qpos / data.qvel; returns the first two balls' positions
    as the reference does."""
    e = restitution if restitution_coeff is None else restitution_coeff
    mu = friction_coefficient if friction is None else friction
    adapter.step_model(model, data, 1, dt, e, mu, 0.0, law="balls", tol=tol)
    q = np.asarray(data.qpos)
    return q[0:3].copy(), q[7:10].copy()


def load_model():
    """models/ball_collision.xml + ball_collision.py:31-34 as (model, data)."""
    return adapter.load_scene_model(scenes.ball_collision())


def main(steps: int = 600):
    model, data = load_model()
    for _ in range(steps):
        step_with_custom_collisions(model, data)
    return np.asarray(data.qpos).reshape(-1, 7)


if __name__ == "__main__":
    print(main())
