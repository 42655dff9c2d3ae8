"""Synthetic scenes C1..C5 and the reference's own model scenes.

Every value is emitted as an explicit float64 array — masses and inertias
are the MuJoCo-compiled constants pinned in SURVEY §8a, not recomputed from
density — so the oracle, the goldens and the HIP path see bit-identical
inputs.  Body order = qpos order (body k at qpos[7k], qvel[6k]).

Sources:
  * models/sphere.xml:10, :27-36   single sphere (C1), dt 0.009
  * models/multi_sphere.xml:10,:27-51 four spheres r 0.1, dt 0.01
  * models/cube.xml:10, :27-36     cube h 0.4 on the 0.7 rad incline, dt 0.009
  * src/config/sim_overrides.py:1-28 restitution / friction per scene
  * src/simulation/single_sphere_bounce.py:40-41 (C1 initial spin)
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Optional

import numpy as np

SPHERE, BOX = 0, 1

# SURVEY §8a scene constants (MuJoCo compiler output for density 50)
M_SPHERE_R01 = 0.20943951023931962
I_SPHERE_R01 = 8.377580409572786e-4
M_SPHERE_R02 = 1.6755160819145563
I_SPHERE_R02 = 0.4 * M_SPHERE_R02 * 0.04
M_CUBE_H04 = 25.600000000000005
I_CUBE_H04 = 2.7306666666666675
INCLINE = 0.7
INCLINE_N = np.array([0.0, -np.sin(INCLINE), np.cos(INCLINE)])   # (0, -0.644217687237691, 0.7648421872844885)
CUBE_Q0 = np.array([np.cos(INCLINE / 2), np.sin(INCLINE / 2), 0.0, 0.0])  # euler="0.7 0 0"
GRAVITY = np.array([0.0, 0.0, -9.8])


@dataclass
class Scene:
    name: str
    kind: np.ndarray          # int32 [N]
    mass: np.ndarray          # f64 [N]
    inertia: np.ndarray       # f64 [N,3]
    size: np.ndarray          # f64 [N,3]
    planes: np.ndarray        # f64 [P,6] normal xyz, point xyz
    qpos0: np.ndarray         # f64 [N,7]
    qvel0: np.ndarray         # f64 [N,6]
    dt: float
    restitution: float
    friction: float
    threshold: float = 0.0
    gravity: np.ndarray = field(default_factory=lambda: GRAVITY.copy())
    normal_convention: str = "oriented"
    names: Optional[list] = None   # body names, for the name-based reference entries

    @property
    def n(self) -> int:
        return int(self.kind.shape[0])

    def params(self) -> dict:
        return dict(dt=self.dt, restitution=self.restitution, friction=self.friction,
                    contact_threshold=self.threshold)

    def with_(self, **kw) -> "Scene":
        return replace(self, **kw)


def _flat_plane() -> np.ndarray:
    return np.array([[0.0, 0.0, 1.0, 0.0, 0.0, 0.0]])


def _incline_plane() -> np.ndarray:
    return np.concatenate([INCLINE_N, np.zeros(3)])[None, :]


def _spheres(n, r, m, inertia):
    return (np.full(n, SPHERE, np.int32), np.full(n, m), np.full((n, 3), inertia),
            np.tile(np.array([r, 0.0, 0.0]), (n, 1)))


def single_sphere() -> Scene:
    """C1 — models/sphere.xml + single_sphere_bounce.py:40-41 (e 1.0, mu 0.5:
    sim_overrides.py:2-8; threshold 0: collision.py:56)."""
    kind, mass, inertia, size = _spheres(1, 0.2, M_SPHERE_R02, I_SPHERE_R02)
    qpos = np.array([[0.0, 0.0, 2.0, 1.0, 0.0, 0.0, 0.0]])
    qvel = np.array([[0.0, 0.0, 0.0, 2.0, 2.0, 0.0]])
    return Scene("single_sphere", kind, mass, inertia, size, _flat_plane(), qpos, qvel,
                 dt=0.009, restitution=1.0, friction=0.5, threshold=0.0, names=["ball"])


def single_cube() -> Scene:
    """models/cube.xml (cube at (0,0,0.4), euler 0.7) + cube_incline.py:46
    (e 0.2, mu 0.6: sim_overrides.py:9-15; threshold 1e-4:
    time_integeration.py:13)."""
    qpos = np.array([[0.0, 0.0, 0.4, *CUBE_Q0]])
    return Scene("single_cube", np.array([BOX], np.int32), np.array([M_CUBE_H04]),
                 np.full((1, 3), I_CUBE_H04), np.full((1, 3), 0.4), _incline_plane(), qpos,
                 np.zeros((1, 6)), dt=0.009, restitution=0.2, friction=0.6, threshold=1e-4,
                 names=["cube"])


def multi_sphere4() -> Scene:
    """models/multi_sphere.xml:30-51 (e 1.0, mu 0.0: sim_overrides.py:22-27)."""
    kind, mass, inertia, size = _spheres(4, 0.1, M_SPHERE_R01, I_SPHERE_R01)
    pos = np.array([[-1.5, -1.5, 2.0], [1.5, -1.5, 2.0], [-1.5, 1.5, 2.0], [1.5, 1.5, 2.0]])
    qpos = np.concatenate([pos, np.tile([1.0, 0, 0, 0], (4, 1))], axis=1)
    return Scene("multi_sphere", kind, mass, inertia, size, _flat_plane(), qpos, np.zeros((4, 6)),
                 dt=0.01, restitution=1.0, friction=0.0, threshold=0.0,
                 names=["ball1", "ball2", "ball3", "ball4"])


def ball_collision(spin: bool = False) -> Scene:
    """models/ball_collision.xml + ball_collision.py:31-34 (two balls r 0.1
    thrown at each other; e 1.0, mu 0.3: sim_overrides.py:16-21; dt 0.01).
    The two-ball contact law (rbhip.World(..., law="balls")).  spin=True:
    a y-offset and initial spins, so the friction and torque terms act."""
    kind, mass, inertia, size = _spheres(2, 0.1, M_SPHERE_R01, I_SPHERE_R01)
    qpos = np.array([[-1.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0], [1.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0]])
    qvel = np.array([[1.0, 0.0, 0.5, 0.0, 0.0, 0.0], [-1.0, 0.0, 0.5, 0.0, 0.0, 0.0]])
    if spin:
        qpos[1, 1] = 0.06
        qvel[0, 3:6] = [0.0, 4.0, 2.0]
        qvel[1, 3:6] = [1.0, -2.0, 0.0]
    return Scene("ball_collision", kind, mass, inertia, size, _flat_plane(), qpos, qvel,
                 dt=0.01, restitution=1.0, friction=0.3, threshold=0.0, names=["ball1", "ball2"])


def balls_pile(nx: int, ny: int, seed: int = 0, spacing: float = 0.25) -> Scene:
    """N-ball generalisation of the two-ball law: an nx*ny grid of r 0.1
    balls dropped from z ~ U(0.3, 1.5) with v_xy ~ N(0, 1), close enough that
    neighbours collide; e 0.9, mu 0.3, dt 0.01."""
    n = nx * ny
    rng = np.random.default_rng(seed)
    kind, mass, inertia, size = _spheres(n, 0.1, M_SPHERE_R01, I_SPHERE_R01)
    iy, ix = np.divmod(np.arange(n), nx)
    qpos = np.zeros((n, 7))
    qpos[:, 0] = (ix - (nx - 1) / 2.0) * spacing
    qpos[:, 1] = (iy - (ny - 1) / 2.0) * spacing
    qpos[:, 2] = rng.uniform(0.3, 1.5, n)
    qpos[:, 3] = 1.0
    qvel = np.zeros((n, 6))
    qvel[:, 0:2] = rng.normal(0.0, 1.0, (n, 2))
    qvel[:, 3:6] = rng.normal(0.0, 3.0, (n, 3))
    return Scene(f"balls_pile_{n}", kind, mass, inertia, size, _flat_plane(), qpos, qvel,
                 dt=0.01, restitution=0.9, friction=0.3, threshold=0.0)


def flat_spheres(nx: int, ny: int, seed: int = 0, spacing: float = 0.3) -> Scene:
    """C2/C3 — nx*ny spheres r 0.1 on flat ground, grid spacing 0.3 (3r),
    z0 ~ U(0.15, 2.0), v_xy ~ N(0, 0.3^2), v_z = 0, w ~ N(0, 2^2);
    e 0.8, mu 0.3, dt 0.01 (multi_sphere.xml:10), threshold 0."""
    n = nx * ny
    rng = np.random.default_rng(seed)
    kind, mass, inertia, size = _spheres(n, 0.1, M_SPHERE_R01, I_SPHERE_R01)
    iy, ix = np.divmod(np.arange(n), nx)
    x = (ix - (nx - 1) / 2.0) * spacing
    y = (iy - (ny - 1) / 2.0) * spacing
    z = rng.uniform(0.15, 2.0, n)
    qpos = np.zeros((n, 7))
    qpos[:, 0], qpos[:, 1], qpos[:, 2], qpos[:, 3] = x, y, z, 1.0
    qvel = np.zeros((n, 6))
    qvel[:, 0:2] = rng.normal(0.0, 0.3, (n, 2))
    qvel[:, 3:6] = rng.normal(0.0, 2.0, (n, 3))
    return Scene(f"flat_spheres_{n}", kind, mass, inertia, size, _flat_plane(), qpos, qvel,
                 dt=0.01, restitution=0.8, friction=0.3, threshold=0.0)


def incline_spheres(nx: int, ny: int, seed: int = 0, spacing: float = 0.3) -> Scene:
    """C4 — spheres r 0.1 resting r + U(0, 0.05) above the 0.7 rad incline
    (normal pinned) on an nx*ny in-plane grid, v = w = 0;
    e 0.2, mu 0.6 (sim_overrides.py:9-15), dt 0.01, threshold 0."""
    n = nx * ny
    rng = np.random.default_rng(seed)
    kind, mass, inertia, size = _spheres(n, 0.1, M_SPHERE_R01, I_SPHERE_R01)
    t1 = np.array([1.0, 0.0, 0.0])
    t2 = np.array([0.0, np.cos(INCLINE), np.sin(INCLINE)])
    iy, ix = np.divmod(np.arange(n), nx)
    u = (ix - (nx - 1) / 2.0) * spacing
    w = (iy - (ny - 1) / 2.0) * spacing
    h = 0.1 + rng.uniform(0.0, 0.05, n)
    pos = u[:, None] * t1 + w[:, None] * t2 + h[:, None] * INCLINE_N
    qpos = np.zeros((n, 7))
    qpos[:, 0:3], qpos[:, 3] = pos, 1.0
    return Scene(f"incline_spheres_{n}", kind, mass, inertia, size, _incline_plane(), qpos,
                 np.zeros((n, 6)), dt=0.01, restitution=0.2, friction=0.6, threshold=0.0)


def _quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def incline_cubes(nx: int, ny: int, seed: int = 0, spacing: float = 3.0) -> Scene:
    """C5 — cubes h 0.4 (m 25.6) posed as cube.xml:33 (0.4 above the in-plane
    grid point, euler 0.7) plus a seeded yaw U(-0.1, 0.1) about the incline
    normal; grid spacing 3.0 > 2*sqrt(3)*h so no cube-cube contact;
    e 0.2, mu 0.6, dt 0.009, threshold 1e-4."""
    n = nx * ny
    rng = np.random.default_rng(seed)
    t1 = np.array([1.0, 0.0, 0.0])
    t2 = np.array([0.0, np.cos(INCLINE), np.sin(INCLINE)])
    iy, ix = np.divmod(np.arange(n), nx)
    u = (ix - (nx - 1) / 2.0) * spacing
    w = (iy - (ny - 1) / 2.0) * spacing
    pos = u[:, None] * t1 + w[:, None] * t2 + np.array([0.0, 0.0, 0.4])
    yaw = rng.uniform(-0.1, 0.1, n)
    qpos = np.zeros((n, 7))
    qpos[:, 0:3] = pos
    for k in range(n):
        qy = np.concatenate([[np.cos(yaw[k] / 2)], np.sin(yaw[k] / 2) * INCLINE_N])
        qpos[k, 3:7] = _quat_mul(qy, CUBE_Q0)
    return Scene(f"incline_cubes_{n}", np.full(n, BOX, np.int32), np.full(n, M_CUBE_H04),
                 np.full((n, 3), I_CUBE_H04), np.full((n, 3), 0.4), _incline_plane(), qpos,
                 np.zeros((n, 6)), dt=0.009, restitution=0.2, friction=0.6, threshold=1e-4)


def box_pile(nx: int, ny: int, layers: int = 3, seed: int = 0, spacing: float = 1.1, h: float = 0.4,
             sphere_every: int = 3) -> Scene:
    """Box-involved contacts (stacking, the Guendelman
    scheme's goal, README.md:18-24): columns of `layers` cubes of
    models/cube.xml's size (half extent 0.4, m 25.6, I 2.7307; other h:
    density 50) on an nx*ny grid with spacing 1.1 (few bounding-sphere
    partners per box at rest), stacked with 0.03 gaps and tilted by up to
    0.2 rad about a random axis, so they land on each other (face-face), lean
    into their neighbours (edge-edge) and topple; every `sphere_every`-th
    column is capped with a sphere r 0.1 (sphere-box).  Flat ground, e 0.2,
    mu 0.6 (sim_overrides.py:9-15), dt 0.005.  Use max_partners=32."""
    rng = np.random.default_rng(seed)
    m_box = M_CUBE_H04 if h == 0.4 else 50.0 * (2 * h) ** 3
    i_box = I_CUBE_H04 if h == 0.4 else m_box * (2 * h) ** 2 / 6.0
    kind, mass, inertia, size, qpos = [], [], [], [], []
    col = 0
    for iy in range(ny):
        for ix in range(nx):
            x = (ix - (nx - 1) / 2.0) * spacing
            y = (iy - (ny - 1) / 2.0) * spacing
            for k in range(layers):
                ax = rng.normal(size=3)
                ax /= np.linalg.norm(ax)
                ang = rng.uniform(0.0, 0.2)
                q = np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * ax])
                z = h + k * (2 * h + 0.03) + rng.uniform(0.0, 0.02)
                kind.append(BOX); mass.append(m_box); inertia.append([i_box] * 3); size.append([h, h, h])
                qpos.append([x + rng.uniform(-0.03, 0.03), y + rng.uniform(-0.03, 0.03), z, *q])
            if sphere_every and col % sphere_every == 0:
                z = h + layers * (2 * h + 0.03) + 0.12
                kind.append(SPHERE); mass.append(M_SPHERE_R01); inertia.append([I_SPHERE_R01] * 3)
                size.append([0.1, 0.0, 0.0]); qpos.append([x + rng.uniform(-0.1, 0.1), y, z, 1.0, 0, 0, 0])
            col += 1
    n = len(kind)
    qvel = np.zeros((n, 6))
    qvel[:, 3:6] = rng.normal(0.0, 0.5, (n, 3))
    return Scene(f"box_pile_{n}", np.array(kind, np.int32), np.array(mass), np.array(inertia), np.array(size),
                 _flat_plane(), np.array(qpos), qvel, dt=0.005, restitution=0.2, friction=0.6, threshold=0.0)


def crowded_cells(nx: int = 10, ny: int = 10, layers: int = 4, seed: int = 0) -> Scene:
    """Broadphase stress (no reference counterpart): one sphere of r 1.0 —
    so cells are 4 m — far off, and nx*ny*layers spheres of r 0.05 (density
    50) in a 0.12-m lattice dropped on flat ground: hundreds of bodies share
    a cell, whose 128-B bucket holds 30 (the rest spill, rb_grid.hpp).
    e 0.3, mu 0.4, dt 0.005."""
    rng = np.random.default_rng(seed)
    n = nx * ny * layers
    m_s = 50.0 * 4.0 / 3.0 * np.pi * 0.05 ** 3
    kind, mass, inertia, size = _spheres(n + 1, 0.05, m_s, 0.4 * m_s * 0.05 ** 2)
    m_b = 50.0 * 4.0 / 3.0 * np.pi
    mass[n], inertia[n], size[n] = m_b, 0.4 * m_b, [1.0, 0.0, 0.0]
    iz, rem = np.divmod(np.arange(n), nx * ny)
    iy, ix = np.divmod(rem, nx)
    qpos = np.zeros((n + 1, 7))
    qpos[:n, 0] = 0.3 + ix * 0.12 + rng.uniform(-0.005, 0.005, n)
    qpos[:n, 1] = 0.3 + iy * 0.12 + rng.uniform(-0.005, 0.005, n)
    qpos[:n, 2] = 0.06 + iz * 0.12 + rng.uniform(0.0, 0.01, n)
    qpos[n, 0:3] = [12.0, 12.0, 1.0]
    qpos[:, 3] = 1.0
    qvel = np.zeros((n + 1, 6))
    qvel[:n, 0:2] = rng.normal(0.0, 0.3, (n, 2))
    return Scene(f"crowded_cells_{n + 1}", kind, mass, inertia, size, _flat_plane(), qpos, qvel,
                 dt=0.005, restitution=0.3, friction=0.4, threshold=0.0)


CONFIGS = {
    # BASELINE.json configs, in order
    "c1": single_sphere,
    "c2": lambda seed=0: flat_spheres(64, 64, seed),
    "c3": lambda seed=0: flat_spheres(256, 256, seed),
    "c4": lambda seed=0: incline_spheres(256, 256, seed),
    "c5": lambda seed=0: incline_cubes(128, 128, seed),
}


def make(name: str, **kw) -> Scene:
    if name in CONFIGS:
        return CONFIGS[name](**kw)
    table = {"single_sphere": single_sphere, "single_cube": single_cube,
             "multi_sphere": multi_sphere4, "ball_collision": ball_collision}
    if name in table:
        return table[name]()
    raise KeyError(f"unknown scene {name!r}; known: {sorted(CONFIGS) + sorted(table)}")


def tiled(scene_fn, world_size: int, shard_nx: int, shard_ny: int, seed: int = 0, **kw) -> Scene:
    """Weak-scaling world: `world_size` patches of shard_nx*shard_ny bodies
    laid side by side in x (one patch per rank, body ids rank-major).  The
    patches share one ground, so bodies near patch seams interact across
    ranks."""
    sc = scene_fn(shard_nx * world_size, shard_ny, seed, **kw)
    n = sc.n
    # scene_fn numbers bodies row-major over (x fastest); regroup so that
    # rank r owns the r-th x-slab: ids rank-major, then row, then column.
    iy, ix = np.divmod(np.arange(n), shard_nx * world_size)
    rank = ix // shard_nx
    order = np.lexsort((ix, iy, rank))
    return replace(sc, name=f"{sc.name}_tiled{world_size}", kind=sc.kind[order],
                   mass=sc.mass[order], inertia=sc.inertia[order], size=sc.size[order],
                   qpos0=sc.qpos0[order], qvel0=sc.qvel0[order])
