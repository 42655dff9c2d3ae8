"""Mirror of src/physics/time_integeration.py (file name kept, sic)."""
import numpy as np

from rbhip import adapter
from src.physics.collision import compute_collision_impulse_friction  # noqa: F401
from src.physics.collision import compute_inertia_tensor_world  # noqa: F401
from src.physics.physics_utils import apply_impulse_friction  # noqa: F401


def timestep_integration(model, obj, data, dt=0.01, restitution=1.0, friction_coeff=0.5,
                         contact_threshold=1e-4):
    """time_integeration.py:13-72 — the same step as
    custom_step_with_impulse_collision_friction with the contact threshold
    defaulting to 1e-4.  Returns the new position (3,)."""
    k = adapter.body_index(model, obj)
    n = len(adapter.free_bodies(model))
    # several free bodies: body k alone steps, its contacts filtered by body
    # (the reference applies every contact to the one body)
    adapter.step_model(model, data, 1, dt, restitution, friction_coeff, contact_threshold,
                       only=k if n > 1 else None)
    qi, _ = adapter.state_index(model)
    return np.array(np.asarray(data.qpos)[qi[k, 0:3]], dtype=np.float64)
