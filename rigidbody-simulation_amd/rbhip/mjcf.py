"""MuJoCo-free loader for the MJCF subset the reference's models use
(SURVEY §8f row 2): models/sphere.xml, cube.xml, multi_sphere.xml and
ball_collision.xml become an rbhip Scene, so the stepper runs headless
without MuJoCo (which stays visualisation-only).

Supported:
  <compiler angle="radian|degree" eulerseq=...>  (MuJoCo default: degree, "xyz")
  <option timestep gravity>                       (defaults 0.002, 0 0 -9.81)
  <default><geom density=...></default>           (top-level class only)
  <worldbody>: static geoms and static bodies (any nesting) carrying planes;
  free bodies (<joint type="free">) with exactly one sphere or box geom at the
  body origin, placed by pos + quat | euler.
Masses and inertias: the MuJoCo-compiled constants SURVEY §8a pins for the
reference's own geoms (sphere r 0.1 / 0.2, cube h 0.4, density 50) — the
closed forms below differ from MuJoCo's compiler in the last bits — and the
closed form (sphere m = rho 4/3 pi r^3, I = 2/5 m r^2; box m = rho 8 hx hy hz,
I_x = m/3 (hy^2 + hz^2) ...) for anything else (parity unpinned).
Plane normals and body quaternions compose elementary rotations, so a
single-axis euler gives (0, -sin a, cos a) and (cos a/2, sin a/2, 0, 0)
exactly (the normal SURVEY §8a pins for cube.xml's incline).
"""
from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET
from typing import Optional

import numpy as np

from .scenes import BOX, SPHERE, Scene

# (geom type, size, density) -> (mass, principal inertia): SURVEY §8a
PINNED = {
    ("sphere", (0.1,), 50.0): (0.20943951023931962, 8.377580409572786e-4),
    ("sphere", (0.2,), 50.0): (1.6755160819145563, 0.4 * 1.6755160819145563 * 0.04),
    ("box", (0.4, 0.4, 0.4), 50.0): (25.600000000000005, 2.7306666666666675),
}
MUJOCO_DEFAULT_DENSITY = 1000.0


def _floats(s: Optional[str], n: Optional[int] = None, default=None):
    if s is None:
        return None if default is None else np.array(default, dtype=np.float64)
    v = np.array([float(t) for t in s.split()], dtype=np.float64)
    if n is not None and v.size != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _rot(axis: int, a: float) -> np.ndarray:
    c, s = math.cos(a), math.sin(a)
    R = np.eye(3)
    i, j = [(1, 2), (0, 2), (0, 1)][axis]
    R[i, i], R[j, j] = c, c
    if axis == 1:
        R[i, j], R[j, i] = s, -s
    else:
        R[i, j], R[j, i] = -s, s
    return R


def _qmul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _qrot(axis: int, a: float) -> np.ndarray:
    q = np.array([math.cos(a / 2), 0.0, 0.0, 0.0])
    q[1 + axis] = math.sin(a / 2)
    return q


class _Frame:
    """Rotation (matrix and quaternion, composed from elementary rotations)
    plus translation."""

    def __init__(self, R=None, q=None, p=None):
        self.R = np.eye(3) if R is None else R
        self.q = np.array([1.0, 0.0, 0.0, 0.0]) if q is None else q
        self.p = np.zeros(3) if p is None else p

    def compose(self, child: "_Frame") -> "_Frame":
        """self * child; identity factors are skipped so exact values survive."""
        eye, q1 = np.eye(3), np.array([1.0, 0.0, 0.0, 0.0])
        rid, cid = np.array_equal(self.R, eye), np.array_equal(child.R, eye)
        R = child.R if rid else (self.R if cid else self.R @ child.R)
        qid, cqid = np.array_equal(self.q, q1), np.array_equal(child.q, q1)
        q = child.q if qid else (self.q if cqid else _qmul(self.q, child.q))
        p = self.p + (child.p if rid else self.R @ child.p)
        return _Frame(R, q, p)


class _Ctx:
    def __init__(self, root: ET.Element):
        comp = root.find("compiler")
        self.degree = comp is None or comp.get("angle", "degree") == "degree"
        self.eulerseq = (comp.get("eulerseq") if comp is not None else None) or "xyz"
        self.density = MUJOCO_DEFAULT_DENSITY
        dflt = root.find("default")
        if dflt is not None and dflt.find("geom") is not None and dflt.find("geom").get("density"):
            self.density = float(dflt.find("geom").get("density"))

    def frame(self, el: ET.Element) -> _Frame:
        p = _floats(el.get("pos"), 3, [0.0, 0.0, 0.0])
        if el.get("quat") is not None:
            q = _floats(el.get("quat"), 4)
            q = q / math.sqrt(float(q @ q))
            w, x, y, z = q
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                          [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                          [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
            return _Frame(R, q, p)
        if el.get("euler") is not None:
            e = _floats(el.get("euler"), 3)
            if self.degree:
                e = e * (math.pi / 180.0)
            R, q = np.eye(3), np.array([1.0, 0.0, 0.0, 0.0])
            seq = self.eulerseq
            for k, ch in enumerate(seq):
                axis = "xyz".index(ch.lower())
                if e[k] == 0.0:
                    continue
                Rk, qk = _rot(axis, float(e[k])), _qrot(axis, float(e[k]))
                if ch.islower():          # intrinsic: rotate about the moving axes
                    R = Rk if np.array_equal(R, np.eye(3)) else R @ Rk
                    q = qk if np.array_equal(q, [1.0, 0, 0, 0]) else _qmul(q, qk)
                else:                     # extrinsic: about the fixed axes
                    R = Rk if np.array_equal(R, np.eye(3)) else Rk @ R
                    q = qk if np.array_equal(q, [1.0, 0, 0, 0]) else _qmul(qk, q)
            return _Frame(R, q, p)
        return _Frame(p=p)


def mass_inertia(gtype: str, size, density: float):
    """(mass, principal inertia[3]) of a sphere / box geom (pinned constants
    for the reference's geoms, closed form otherwise)."""
    key = (gtype, tuple(float(s) for s in size), float(density))
    if key in PINNED:
        m, i = PINNED[key]
        return m, np.full(3, i)
    if gtype == "sphere":
        r = float(size[0])
        m = density * (4.0 / 3.0) * math.pi * r ** 3
        return m, np.full(3, 0.4 * m * r * r)
    hx, hy, hz = (float(s) for s in size)
    m = density * 8.0 * hx * hy * hz
    return m, np.array([m / 3 * (hy * hy + hz * hz), m / 3 * (hx * hx + hz * hz), m / 3 * (hx * hx + hy * hy)])


def load(source: str, restitution: float = 1.0, friction: float = 0.5, threshold: float = 0.0,
         name: Optional[str] = None) -> Scene:
    """Scene from an MJCF file path or XML string.  restitution / friction /
    threshold are the step parameters the calling script passes (the MJCF
    friction/solref attributes belong to MuJoCo's own solver, unused here)."""
    text = open(source).read() if os.path.exists(source) else source
    root = ET.fromstring(text)
    if root.tag != "mujoco":
        raise ValueError("not an MJCF document (<mujoco> root expected)")
    ctx = _Ctx(root)
    opt = root.find("option")
    dt = float(opt.get("timestep", "0.002")) if opt is not None else 0.002
    gravity = _floats(opt.get("gravity") if opt is not None else None, 3, [0.0, 0.0, -9.81])
    wb = root.find("worldbody")
    if wb is None:
        raise ValueError("MJCF without <worldbody>")
    planes, bodies = [], []

    def add_plane(g: ET.Element, parent: _Frame):
        f = parent.compose(ctx.frame(g))
        planes.append(np.concatenate([f.R[:, 2], f.p]))

    def walk(el: ET.Element, parent: _Frame):
        for g in el.findall("geom"):
            if g.get("type", "sphere") == "plane":
                add_plane(g, parent)
            elif el is not wb and el.find("joint") is None:
                raise NotImplementedError(f"static non-plane geom {g.get('name')!r}")
        for b in el.findall("body"):
            f = parent.compose(ctx.frame(b))
            joints = b.findall("joint") + b.findall("freejoint")
            free = any(j.tag == "freejoint" or j.get("type") == "free" for j in joints)
            if not free:
                if joints:
                    raise NotImplementedError(f"body {b.get('name')!r}: only free joints are supported")
                walk(b, f)
                continue
            if b.findall("body"):
                raise NotImplementedError(f"free body {b.get('name')!r} with child bodies")
            geoms = b.findall("geom")
            if len(geoms) != 1 or geoms[0].get("type", "sphere") not in ("sphere", "box"):
                raise NotImplementedError(f"free body {b.get('name')!r}: exactly one sphere or box geom")
            g = geoms[0]
            if np.any(_floats(g.get("pos"), 3, [0.0, 0.0, 0.0]) != 0.0):
                raise NotImplementedError(f"free body {b.get('name')!r}: geom must sit at the body origin")
            gtype = g.get("type", "sphere")
            size = _floats(g.get("size"))
            size = size[:1] if gtype == "sphere" else size[:3]
            if g.get("mass") is not None:         # explicit mass: inertia scales with it
                m = float(g.get("mass"))
                m_unit, i_unit = mass_inertia(gtype, size, 1.0)
                inertia = i_unit * (m / m_unit)
            else:
                m, inertia = mass_inertia(gtype, size, float(g.get("density", ctx.density)))
            bodies.append((b.get("name"), SPHERE if gtype == "sphere" else BOX, m, inertia,
                           np.array([size[0], 0.0, 0.0]) if gtype == "sphere" else size.copy(), f))
    walk(wb, _Frame())
    if not bodies:
        raise ValueError("MJCF has no free bodies")
    n = len(bodies)
    qpos = np.zeros((n, 7))
    for k, (_, _, _, _, _, f) in enumerate(bodies):
        qpos[k, 0:3], qpos[k, 3:7] = f.p, f.q
    if name is None:
        name = os.path.splitext(os.path.basename(source))[0] if os.path.exists(source) else "mjcf"
    return Scene(name, np.array([b[1] for b in bodies], np.int32), np.array([b[2] for b in bodies], np.float64),
                 np.stack([b[3] for b in bodies]).astype(np.float64), np.stack([b[4] for b in bodies]),
                 np.array(planes, np.float64).reshape(-1, 6), qpos, np.zeros((n, 6)), dt=dt,
                 restitution=restitution, friction=friction, threshold=threshold, gravity=gravity,
                 names=[b[0] for b in bodies])


__all__ = ["load", "mass_inertia", "PINNED"]
