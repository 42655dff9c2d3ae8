"""rbhip — host package of the MI355X-native rigid-body stepper.

Import path: put `<repo>/rigidbody-simulation_amd` on sys.path (the same
way the reference puts its repo root on PYTHONPATH for `src.*`).

  rbhip.World        a scene resident on one GPU (librbhip.so via ctypes)
  rbhip.scenes       synthetic scenes C1..C5 and the reference model scenes
  rbhip.shard        body-range sharding over torch.distributed
  rbhip.mjcf         MuJoCo-free loader for the reference's models/*.xml
  rbhip.sampling     host-side sampling of a GPU-resident run
"""
from . import scenes  # noqa: F401
from ._lib import RbError, load  # noqa: F401
from .world import World, kat_apply, kat_impulse, kat_inertia, kat_narrow, kat_pair_impulse  # noqa: F401

__all__ = ["World", "RbError", "load", "scenes", "kat_impulse", "kat_inertia", "kat_apply", "kat_pair_impulse",
           "kat_narrow"]
