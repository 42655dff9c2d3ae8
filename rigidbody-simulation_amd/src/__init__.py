"""Drop-in mirror of the reference's `src` package surface (hot path only).

`src.physics.collision`, `src.physics.physics_utils`,
`src.physics.time_integeration` and `src.simulation.multi_sphere_bounce`
keep the reference's names, signatures, argument meaning and return types;
the arithmetic runs in librbhip.so on the GPU (no CPU fallback).
Put `<repo>/rigidbody-simulation_amd` on sys.path, as the reference puts its
repo root there.
"""
