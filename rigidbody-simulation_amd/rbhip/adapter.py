"""Model/data adapter for the reference's step-function signatures.

The reference step functions take MuJoCo's (model, data) and mutate
data.qpos / data.qvel in place (collision.py:97-100,
time_integeration.py:67-70, multi_sphere_bounce.py:85-88).  Here `model`
is either

  * a SceneModel (duck-typed MjModel built from an rbhip Scene or from the
    MJCF loader, rbhip.mjcf) — the MuJoCo-free path, or
  * a real mujoco.MjModel, when MuJoCo is installed for visualisation only
    (read: body masses/inertias, free joints, plane/sphere/box geoms).

The world (device state) is cached per model; every call uploads data's
state, steps on the GPU and writes the result back into data, as the
reference does per frame.
"""
from __future__ import annotations

import warnings
import weakref
from typing import Optional

import numpy as np

from .scenes import BOX, GRAVITY, SPHERE, Scene
from .world import World


class _Opt:
    def __init__(self, timestep: float, gravity):
        self.timestep = float(timestep)
        self.gravity = np.array(gravity, dtype=np.float64)


class SceneModel:
    """Duck-typed MjModel: body 0 = world, body 1 = the static plane body,
    bodies 2.. = the free bodies (the order of models/sphere.xml, cube.xml)."""

    FIRST = 2

    def __init__(self, scene: Scene, names: Optional[list] = None):
        self.rb_scene = scene
        n = scene.n
        self.nbody = n + self.FIRST
        self.body_mass = np.zeros(self.nbody)
        self.body_inertia = np.zeros((self.nbody, 3))
        self.body_mass[self.FIRST:] = scene.mass
        self.body_inertia[self.FIRST:] = scene.inertia
        self.opt = _Opt(scene.dt, scene.gravity)
        names = names or scene.names or [f"body{k}" for k in range(n)]
        self.names = ["world", "plane_body"] + list(names)
        self.nq, self.nv = 7 * n, 6 * n

    def name2id(self, name: str) -> int:
        try:
            return self.names.index(name)
        except ValueError:
            return -1


class SceneData:
    """Duck-typed MjData: qpos [7N], qvel [6N], xfrc_applied [nbody, 6], time."""

    def __init__(self, model: SceneModel):
        sc = model.rb_scene
        self.qpos = sc.qpos0.reshape(-1).copy()
        self.qvel = sc.qvel0.reshape(-1).copy()
        self.xfrc_applied = np.zeros((model.nbody, 6))
        self.time = 0.0
        self.ncon = 0


def _mujoco():
    import mujoco
    return mujoco


def free_bodies(model) -> list:
    """Body ids of the free bodies, in body order.  SceneModel: bodies
    FIRST..nbody-1; a MuJoCo model: every body whose single joint is a free
    joint (body_jntnum / body_jntadr / jnt_type)."""
    if isinstance(model, SceneModel):
        return list(range(SceneModel.FIRST, model.nbody))
    mj = _mujoco()
    return [b for b in range(model.nbody) if model.body_jntnum[b] == 1 and
            model.jnt_type[model.body_jntadr[b]] == mj.mjtJoint.mjJNT_FREE]


def state_index(model):
    """(qpos index [nfree, 7], qvel index [nfree, 6]) of the free bodies'
    joints: jnt_qposadr / jnt_dofadr for a MuJoCo model (joints need not be
    contiguous or start at 0), stride 7 / 6 for a SceneModel."""
    fb = free_bodies(model)
    if isinstance(model, SceneModel):
        k = np.arange(len(fb))
        return 7 * k[:, None] + np.arange(7), 6 * k[:, None] + np.arange(6)
    qa = np.array([model.jnt_qposadr[model.body_jntadr[b]] for b in fb], dtype=np.int64)
    da = np.array([model.jnt_dofadr[model.body_jntadr[b]] for b in fb], dtype=np.int64)
    return qa[:, None] + np.arange(7), da[:, None] + np.arange(6)


def scene_from_mujoco(model, restitution: float = 1.0, friction: float = 0.5) -> Scene:
    """Scene from a compiled mujoco.MjModel (free bodies with one sphere or
    box geom each; planes on static bodies).  restitution / friction are the
    scene's defaults only — every step call passes the caller's values
    (collision.py:56-61).  Parity of this path is unpinned: MuJoCo is not
    installed in the build container (tested with a duck-typed fake)."""
    mj = _mujoco()
    d = mj.MjData(model)
    mj.mj_forward(model, d)
    free = free_bodies(model)
    kind, size = [], []
    planes = []
    for g in range(model.ngeom):
        t = model.geom_type[g]
        if t == mj.mjtGeom.mjGEOM_PLANE:
            mat = np.asarray(d.geom_xmat[g]).reshape(3, 3)
            planes.append(np.concatenate([mat[:, 2], d.geom_xpos[g]]))
    for b in free:
        gs = [g for g in range(model.ngeom) if model.geom_bodyid[g] == b]
        if len(gs) != 1 or model.geom_type[gs[0]] not in (mj.mjtGeom.mjGEOM_SPHERE, mj.mjtGeom.mjGEOM_BOX):
            raise NotImplementedError("each free body must carry exactly one sphere or box geom")
        g = gs[0]
        kind.append(SPHERE if model.geom_type[g] == mj.mjtGeom.mjGEOM_SPHERE else BOX)
        size.append(np.asarray(model.geom_size[g], dtype=np.float64).copy())
    qi, vi = state_index(model)
    qpos = np.asarray(d.qpos, dtype=np.float64)[qi]
    qvel = np.asarray(d.qvel, dtype=np.float64)[vi]
    return Scene("mujoco", np.array(kind, np.int32), np.asarray(model.body_mass, np.float64)[free].copy(),
                 np.asarray(model.body_inertia, np.float64)[free].copy(), np.array(size),
                 np.array(planes, dtype=np.float64).reshape(-1, 6), qpos, qvel,
                 dt=float(model.opt.timestep), restitution=float(restitution), friction=float(friction),
                 gravity=np.array(model.opt.gravity, dtype=np.float64))


_worlds: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_worlds_by_id: dict = {}


def _scene_of(model, restitution: float = 1.0, friction: float = 0.5) -> Scene:
    sc = getattr(model, "rb_scene", None)
    return sc if sc is not None else scene_from_mujoco(model, restitution, friction)


def world_for(model, normal_convention: str = "oriented", law: str = "mujoco", tol: float = 0.01,
              restitution: float = 1.0, friction: float = 0.5) -> World:
    """The cached GPU world of `model` (one per model and contact law)."""
    try:
        ws = _worlds.get(model)
    except TypeError:
        ws = _worlds_by_id.get(id(model))
    if ws is None:
        ws = {}
        try:
            _worlds[model] = ws
        except TypeError:
            _worlds_by_id[id(model)] = ws
    w = ws.get(law)
    if w is None:
        w = ws[law] = World(_scene_of(model, restitution, friction), normal_convention=normal_convention,
                            law=law, tol=tol)
    elif law == "balls" and w.tol != tol:
        w.set_contact_law(law, tol)
    return w


def name2id(model, obj: str) -> int:
    """mj_name2id(model, mjOBJ_BODY, obj): the SceneModel's own table, or
    mujoco.mj_name2id for a real MjModel (collision.py:58)."""
    if isinstance(model, SceneModel) or not hasattr(model, "body_jntnum"):
        return model.name2id(obj) if hasattr(model, "name2id") else -1
    mj = _mujoco()
    return int(mj.mj_name2id(model, mj.mjtObj.mjOBJ_BODY, obj))


def body_index(model, obj: str) -> int:
    """mj_name2id(model, mjOBJ_BODY, obj) -> free-body index.  The reference
    indexes model arrays with the raw id, so an unknown name (-1) selects the
    LAST body (single_sphere_bounce.py:67 passes "sphere" for the
    body "ball" and works by accident); reproduced, with a warning."""
    bid = name2id(model, obj)
    if bid < 0:
        warnings.warn(f"body {obj!r} not found: using the last body, as mj_name2id's -1 does "
                      f"in the reference (SURVEY D4)", stacklevel=3)
        bid = model.nbody - 1
    fb = free_bodies(model)
    if bid not in fb:
        raise ValueError(f"body {obj!r} is not a free body")
    return fb.index(bid)


def step_model(model, data, nsteps: int, dt: float, restitution: float, friction: float,
               threshold: float, normal_convention: str = "oriented", law: str = "mujoco",
               tol: float = 0.01, only: Optional[int] = None) -> None:
    """Upload data's state, run nsteps reference steps on the GPU, write back
    (the free bodies' joints only, at their jnt_qposadr / jnt_dofadr).

    only = k: the single-body entries on a scene of several free bodies
    (time_integeration.py:13-72, collision.py:56-102; SURVEY D11 "with N
    bodies, filter by body"): one step of free body k alone — its gravity,
    its own contacts (planes, then partners by ascending id, the partners
    static at their step-start positions) and its integration; every other
    body stays where it is.  The device steps every body (a step is Jacobi
    across bodies, so the others' results never feed body k's) and only
    body k's rows are written back: an owned-body mask at the boundary."""
    w = world_for(model, normal_convention, law, tol, restitution, friction)
    qi, vi, fb, contiguous = _layout(model, w)
    qpos, qvel = np.asarray(data.qpos), np.asarray(data.qvel)
    n = fb.shape[0]
    if only is not None:
        if not 0 <= only < n:
            raise ValueError(f"free body {only} out of range (0..{n - 1})")
        if nsteps != 1:
            raise ValueError("a single-body step is one reference step")
        w.set_state(qpos[qi], qvel[vi])
        w.set_xfrc(_applied(data, fb))
        w.step(1, dt=dt, restitution=restitution, friction=friction, threshold=threshold)
        q, v = w.get_state()
        data.qpos[qi[only]] = q[only]
        data.qvel[vi[only]] = v[only]
        return
    contiguous = contiguous and all(isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous
                                    for a in (data.qpos, data.qvel))
    if contiguous:                  # free joints at qpos[0:7n] / qvel[0:6n]: views, no gathers
        w.set_state(qpos[:7 * n].reshape(n, 7), qvel[:6 * n].reshape(n, 6))
    else:
        w.set_state(qpos[qi], qvel[vi])
    w.set_xfrc(_applied(data, fb))
    w.step(nsteps, dt=dt, restitution=restitution, friction=friction, threshold=threshold)
    if contiguous:
        w.get_state(data.qpos[:7 * n].reshape(n, 7), data.qvel[:6 * n].reshape(n, 6))
    else:
        q, v = w.get_state()
        data.qpos[qi] = q
        data.qvel[vi] = v


def _applied(data, fb):
    """The free bodies' applied forces (collision.py:66-70), or None when
    all zero: the common all-zero array is told by one contiguous scan,
    without gathering the free bodies' rows."""
    xf = getattr(data, "xfrc_applied", None)
    if xf is None:
        return None
    xf = np.asarray(xf)
    if xf.shape[0] <= fb[-1] or _all_zero(xf):
        return None
    xf_free = xf[fb]
    return xf_free if np.any(xf_free) else None


def _all_zero(a: np.ndarray) -> bool:
    """not a.any(), fast for the common all-+0.0 float64 array: the largest
    64-bit word is 0 only then (one integer max, ~10x faster than any() on
    65,537 x 6); anything else (a -0.0, a force) decided by any()."""
    if a.dtype == np.float64 and a.flags.c_contiguous and a.size:
        if int(a.reshape(-1).view(np.uint64).max()) == 0:
            return True
    return not a.any()


def _layout(model, w: World):
    """(qpos index, qvel index, free body ids, contiguous) of a model, cached
    on its world: the per-frame entry pays no O(N) Python work for them
    (65,536 bodies: 15.7 ms per call before, measured on MI355X)."""
    lay = getattr(w, "_adapter_layout", None)
    if lay is None:
        qi, vi = state_index(model)
        fb = np.asarray(free_bodies(model), dtype=np.int64)
        n = fb.shape[0]
        contiguous = (np.array_equal(qi, 7 * np.arange(n)[:, None] + np.arange(7)) and
                      np.array_equal(vi, 6 * np.arange(n)[:, None] + np.arange(6)))
        lay = w._adapter_layout = (qi, vi, fb, contiguous)
    return lay


def load_scene_model(scene: Scene):
    """(SceneModel, SceneData) for a Scene — what MjModel.from_xml_path +
    MjData give the reference scripts."""
    m = SceneModel(scene)
    return m, SceneData(m)


__all__ = ["SceneModel", "SceneData", "world_for", "step_model", "body_index", "load_scene_model",
           "scene_from_mujoco", "free_bodies", "state_index", "name2id", "GRAVITY"]
