"""Host-side sampling of a GPU-resident run: the caller
side of the boundary.  The reference records every body's position every
frame (mujoco_viewer.py:113-119, multi_sphere_bounce.py:90); here the world
steps on the device in graph-replayed chunks and the state crosses PCIe only
every `every` steps."""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .world import World


def run_sampled(world: World, nsteps: int, every: int,
                on_sample: Callable[[int, float, np.ndarray, np.ndarray], None],
                t0: float = 0.0, dt: Optional[float] = None, **params) -> float:
    """Advance `world` by nsteps reference steps, calling
    on_sample(step, time, qpos, qvel) after every `every` steps (and after the
    last one).  Returns the simulation time reached."""
    if every < 1:
        raise ValueError("every must be >= 1")
    dt = world.scene.dt if dt is None else dt
    done, t = 0, t0
    while done < nsteps:
        k = min(every, nsteps - done)
        world.step(k, dt=dt, **params)
        done += k
        t = t0 + done * dt
        q, v = world.get_state()
        on_sample(done, t, q, v)
    return t


__all__ = ["run_sampled"]
