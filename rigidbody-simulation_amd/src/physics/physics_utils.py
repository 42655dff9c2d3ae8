"""Mirror of src/physics/physics_utils.py, evaluated on the GPU."""
import numpy as np

from rbhip import kat_apply


def apply_impulse_friction(vel, omega, mass, inertia_world, contact_point, normal, jn, jt):
    """physics_utils.py:25-49: Δv = (jn·n + jt)/m, Δω = inv(I_w)(r × (jn·n + jt)).
    Returns new (vel, omega) arrays, as the reference does.  Accepts single
    3-vectors or batches (leading dimension B)."""
    v = np.asarray(vel, np.float64)
    single = v.ndim == 1
    v = v.reshape(-1, 3)
    B = v.shape[0]
    row = np.zeros((B, 26))
    row[:, 0] = np.broadcast_to(np.asarray(mass, np.float64), (B,))
    row[:, 1:4] = v
    row[:, 4:7] = np.broadcast_to(np.asarray(omega, np.float64).reshape(-1, 3), (B, 3))
    row[:, 7:10] = np.broadcast_to(np.asarray(contact_point, np.float64).reshape(-1, 3), (B, 3))
    row[:, 10:13] = np.broadcast_to(np.asarray(normal, np.float64).reshape(-1, 3), (B, 3))
    row[:, 13] = np.broadcast_to(np.asarray(jn, np.float64).reshape(-1), (B,))
    row[:, 14:17] = np.broadcast_to(np.asarray(jt, np.float64).reshape(-1, 3), (B, 3))
    row[:, 17:26] = np.broadcast_to(np.asarray(inertia_world, np.float64).reshape(-1, 9), (B, 9))
    out = kat_apply(row)
    if single:
        return out[0, 0:3].copy(), out[0, 3:6].copy()
    return out[:, 0:3].copy(), out[:, 3:6].copy()
