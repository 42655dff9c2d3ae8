"""Mirror of src/physics/collision.py, evaluated on the GPU (librbhip.so)."""
import numpy as np

from rbhip import adapter, kat_impulse, kat_inertia
from src.physics.physics_utils import apply_impulse_friction  # noqa: F401  (same import shape)


def _rows(mass, inertia_world, vel, omega, contact_point, normal, restitution, friction_coeff):
    v = np.asarray(vel, np.float64)
    single = v.ndim == 1
    v = v.reshape(-1, 3)
    B = v.shape[0]
    row = np.zeros((B, 24))
    row[:, 0] = np.broadcast_to(np.asarray(mass, np.float64), (B,))
    row[:, 1] = restitution
    row[:, 2] = friction_coeff
    row[:, 3:6] = v
    row[:, 6:9] = np.broadcast_to(np.asarray(omega, np.float64).reshape(-1, 3), (B, 3))
    row[:, 9:12] = np.broadcast_to(np.asarray(contact_point, np.float64).reshape(-1, 3), (B, 3))
    row[:, 12:15] = np.broadcast_to(np.asarray(normal, np.float64).reshape(-1, 3), (B, 3))
    Iw = np.eye(3) if inertia_world is None else np.asarray(inertia_world, np.float64)
    row[:, 15:24] = np.broadcast_to(Iw.reshape(-1, 9), (B, 9))
    return row, single


def compute_collision_impulse_friction(mass, inertia_world, vel, omega, contact_point, normal,
                                       restitution, friction_coeff):
    """collision.py:7-48 — normal impulse jn and Coulomb friction impulse jt of
    a body against a static surface (inertia_world is unused, as in the
    reference).  Returns (jn, jt) with jn a float and jt an ndarray(3); for a
    batch (leading dimension B), (jn[B], jt[B,3])."""
    row, single = _rows(mass, inertia_world, vel, omega, contact_point, normal, restitution,
                        friction_coeff)
    out = kat_impulse(row)
    if single:
        return float(out[0, 0]), out[0, 1:4].copy()
    return out[:, 0].copy(), out[:, 1:4].copy()


def compute_inertia_tensor_world(inertia_diag, q):
    """collision.py:51-53 — R(q) diag(I) R^T (q in MuJoCo's wxyz order)."""
    row = np.concatenate([np.asarray(inertia_diag, np.float64).reshape(3),
                          np.asarray(q, np.float64).reshape(4)])
    return kat_inertia(row[None, :])[0, 0:9].reshape(3, 3)


def custom_step_with_impulse_collision_friction(model, obj, data, dt=0.01, restitution=1.0,
                                                friction_coeff=1.0, contact_threshold=0):
    """collision.py:56-102 — one step of the single free body `obj`: contacts
    (mj_forward's role), gravity, Gauss-Seidel impulses with friction over
    the contacts with dist < 0 and |dist| >= contact_threshold, semi-implicit
    integration.  Mutates data.qpos[0:7] / data.qvel[0:6]; returns the new
    position (3,)."""
    k = adapter.body_index(model, obj)
    n = len(adapter.free_bodies(model))
    # several free bodies: body k alone steps, its contacts filtered by body
    # (the reference applies every contact to the one body)
    adapter.step_model(model, data, 1, dt, restitution, friction_coeff, contact_threshold,
                       only=k if n > 1 else None)
    qi, _ = adapter.state_index(model)
    return np.array(np.asarray(data.qpos)[qi[k, 0:3]], dtype=np.float64)
