"""MuJoCo-free MJCF loader: the reference's own models
load to exactly the scenes the goldens pin (SURVEY §8a constants), and the
supported subset parses as MuJoCo would.  CPU only."""
import math
import os

import numpy as np
import pytest

from rbhip import mjcf, scenes

REF_MODELS = "/root/reference/models"


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference checkout not present")
@pytest.mark.parametrize("model,scene", [("sphere", scenes.single_sphere), ("cube", scenes.single_cube),
                                         ("multi_sphere", scenes.multi_sphere4)])
def test_reference_models_match_pinned_scenes(model, scene):
    sc, ref = mjcf.load(os.path.join(REF_MODELS, model + ".xml")), scene()
    for f in ("kind", "mass", "inertia", "size", "planes", "gravity"):
        assert np.array_equal(getattr(sc, f), getattr(ref, f)), f
    assert np.array_equal(sc.qpos0, ref.qpos0) or model == "sphere"   # C1 adds the initial spin only
    assert np.array_equal(sc.qpos0[:, :3], ref.qpos0[:, :3])
    assert sc.dt == ref.dt and sc.names == ref.names


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference checkout not present")
def test_ball_collision_model():
    sc = mjcf.load(os.path.join(REF_MODELS, "ball_collision.xml"))
    assert sc.n == 2 and sc.names == ["ball1", "ball2"]
    assert np.array_equal(sc.qpos0[:, :3], [[-1.0, 0.0, 1.0], [1.0, 0.0, 1.0]])
    assert sc.mass[0] == scenes.M_SPHERE_R01 and sc.dt == 0.01


XML = """<mujoco>
  <compiler angle="degree"/>
  <default><geom density="200"/></default>
  <option timestep="0.005"/>
  <worldbody>
    <body name="ramp" pos="0 0 1"><body name="inner" euler="0 0 90">
      <geom type="plane" size="1 1 0.1" euler="30 0 0" pos="1 0 0"/></body></body>
    <body name="a" pos="1 2 3" quat="0 1 0 0"><freejoint/><geom type="sphere" size="0.25"/></body>
    <body name="b" pos="0 0 1"><joint type="free"/><geom type="box" size="0.1 0.2 0.3" mass="2"/></body>
  </worldbody>
</mujoco>"""


def test_inline_subset():
    sc = mjcf.load(XML, restitution=0.5, friction=0.2)
    assert sc.dt == 0.005 and np.array_equal(sc.gravity, [0.0, 0.0, -9.81])   # MuJoCo defaults
    assert sc.names == ["a", "b"] and list(sc.kind) == [scenes.SPHERE, scenes.BOX]
    m_a = 200 * 4 / 3 * math.pi * 0.25 ** 3
    assert sc.mass[0] == pytest.approx(m_a, rel=1e-15)
    assert np.allclose(sc.inertia[0], 0.4 * m_a * 0.0625, rtol=1e-15)
    assert sc.mass[1] == 2.0
    assert np.allclose(sc.inertia[1], [2 / 3 * (0.04 + 0.09), 2 / 3 * (0.01 + 0.09), 2 / 3 * (0.01 + 0.04)])
    assert np.array_equal(sc.qpos0[0], [1, 2, 3, 0, 1, 0, 0])
    # plane: Rz(90) then Rx(30) about the moving axes, at ramp + Rz(90)(1, 0, 0)
    n = np.array([math.sin(math.pi / 6) * math.sin(math.pi / 2), -math.sin(math.pi / 6) * math.cos(math.pi / 2),
                  math.cos(math.pi / 6)])
    assert np.allclose(sc.planes[0, :3], n, atol=1e-15)
    assert np.allclose(sc.planes[0, 3:], [0.0, 1.0, 1.0], atol=1e-15)
    assert sc.restitution == 0.5 and sc.friction == 0.2


@pytest.mark.parametrize("body", [
    '<body><joint type="hinge"/><geom type="sphere" size="0.1"/></body>',
    '<body><freejoint/><geom type="capsule" size="0.1 0.2"/></body>',
    '<body><freejoint/><geom type="sphere" size="0.1" pos="0 0 1"/></body>',
])
def test_unsupported_rejected(body):
    with pytest.raises(NotImplementedError):
        mjcf.load(f"<mujoco><worldbody>{body}</worldbody></mujoco>")
